# bench.py's own hardware-queue setting on a box that exports GPU_MAX_HW_QUEUES=4: five frames in flight on
# quarter grids (the tiled shape) at N = 1 with PT_BENCH_HW_QUEUES 4 and 8, then the default line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hwqb
echo "box GPU_MAX_HW_QUEUES=$GPU_MAX_HW_QUEUES"
for q in 4 8; do
  PT_BENCH_HW_QUEUES=$q PT_BENCH_INFLIGHT=5 PT_BENCH_GRID_SHARE=25 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hwqb/f5_q$q.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('F=5 S=25 Q', c['hw_queues'], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame')" gpurun_out/hwqb/f5_q$q.json
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hwqb/default.json 2>/dev/null || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('default F', c['frames_in_flight'], 'Q', c['hw_queues'], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame')" gpurun_out/hwqb/default.json
