# Round-4 multi-frame launches (pt_render_frames): the whole -m gpu suite, the default kernel against the
# previous commit's build (lib_prev: the refill restructured around LANE_GEN), then rank 0's 8/4/2-way share
# and the whole frame with G frames per launch (tools/tile_scaling.py --group; ms per frame).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_group.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
TAG=${1:-group}
mkdir -p gpurun_out/$TAG
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
  tail -2 gpurun_out/$TAG/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
fi
one() {  # name libdir workload
  env PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$2 timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline > gpurun_out/$TAG/$1_$3.json 2> gpurun_out/$TAG/$1_$3.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" gpurun_out/$TAG/$1_$3.json "$1" "$3" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  one new_$r lib metric
  one prev_$r lib_prev metric
done
run() {  # name env... (ARGS: tile_scaling arguments)
  n=$1; shift
  env "$@" timeout -k 10 200 python tools/tile_scaling.py $ARGS > gpurun_out/$TAG/$n.txt 2>&1 || exit $?
  echo "$n $(tail -1 gpurun_out/$TAG/$n.txt)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  ARGS="--counts 8 --ranks-max 1 --frames 24 --inflight 5 --share 25" run s8_g1_f5_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --frames 6 --inflight 3 --share 50 --group 4" run s8_g4_f3_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --frames 6 --inflight 3 --share 45 --group 4" run s8_g4_f3s45_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --frames 6 --inflight 2 --share 100 --group 4" run s8_g4_f2_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --frames 4 --inflight 3 --share 50 --group 8" run s8_g8_f3_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --frames 24 --inflight 5 --share 25" run s4_g1_f5_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --frames 6 --inflight 3 --share 50 --group 4" run s4_g4_f3_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --frames 8 --inflight 3 --share 50 --group 2" run s4_g2_f3_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --frames 24 --inflight 5 --share 25" run s2_g1_f5_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --frames 8 --inflight 3 --share 50 --group 2" run s2_g2_f3_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --frames 6 --inflight 3 --share 50 --group 4" run s2_g4_f3_$r PT_TRI_MIN=3
done
for g in 1 4; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/$TAG/pmc_s8_g$g -o run -- python3 tools/share_render.py --n 8 --group $g > gpurun_out/$TAG/pmc_s8_g$g.log 2>&1 || exit $?
  grep "share 0" gpurun_out/$TAG/pmc_s8_g$g.log | tee -a gpurun_out/$TAG/summary.txt
done
echo done
