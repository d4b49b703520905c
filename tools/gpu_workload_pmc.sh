# VALU and HBM counters of the pass kernel on the heavier configurations (one frame in flight), separate passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/wlpmc
for wl in c3 c4 c5; do
  P="python3 bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline"
  PT_BENCH_INFLIGHT=1 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/wlpmc/$wl/sq -o run -- $P > gpurun_out/wlpmc/$wl.json 2> gpurun_out/wlpmc/$wl.sq.err || exit $?
  PT_BENCH_INFLIGHT=1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/wlpmc/$wl/fetch -o run -- $P > /dev/null 2> gpurun_out/wlpmc/$wl.f.err || exit $?
  PT_BENCH_INFLIGHT=1 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/wlpmc/$wl/write -o run -- $P > /dev/null 2> gpurun_out/wlpmc/$wl.w.err || exit $?
  echo "== $wl $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], 'Mrays/s', r['avg_launch_ms'], 'ms/launch', r['kernel'])" gpurun_out/wlpmc/$wl.json)"
  python3 tools/pmc_summary.py gpurun_out/wlpmc/$wl | grep -A8 pass_kernel_u
done
