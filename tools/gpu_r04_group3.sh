# Round-4 frame groups, final check: the whole -m gpu suite and smoke(), the N = 1 bench line, the N > 1 bench
# rehearsal with gloo on one GPU (groups on by default at N > 1), then rank 0's share per frame over the
# bench's own timed sequence (20 frames: launches of at most G frames) for the bench defaults and the
# one-frame-per-launch setting.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_group3.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-group3}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cut -c1-220 gpurun_out/$TAG/bench.json
bash tools/gpu_multirank_rehearsal.sh $TAG/mr || exit $?
export GPU_MAX_HW_QUEUES=16
run() {  # name env... (ARGS: tile_scaling arguments)
  n=$1; shift
  env "$@" timeout -k 10 200 python tools/tile_scaling.py $ARGS > gpurun_out/$TAG/$n.txt 2>&1 || exit $?
  echo "$n $(tail -1 gpurun_out/$TAG/$n.txt)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  ARGS="--counts 8 --ranks-max 1 --frames 20 --inflight 5 --share 25" run s8_g1_f5_t20_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run s8_g8_f2_t20_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --total 20 --inflight 3 --share 50 --group 4" run s8_g4_f3_t20_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --total 40 --inflight 2 --share 100 --group 8" run s8_g8_f2_t40_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --frames 20 --inflight 5 --share 25" run s4_g1_f5_t20_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --total 20 --inflight 3 --share 50 --group 8" run s4_g8_f3_t20_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run s4_g8_f2_t20_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --frames 20 --inflight 5 --share 25" run s2_g1_f5_t20_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --total 20 --inflight 3 --share 50 --group 4" run s2_g4_f3_t20_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 4" run s2_g4_f2_t20_$r PT_TRI_MIN=3
done
echo done
