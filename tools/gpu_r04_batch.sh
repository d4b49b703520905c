# Round-4 experiment: what one launch over several frames would buy. Rank 0's 8-way share and the whole frame,
# rendered 8 passes per launch (the bench) or 32 passes per launch (PT_PASS_BATCH=32, four frames' worth of
# units in one launch), under frames in flight; ms per 8 passes (tools/tile_scaling.py --spp).
#   gpurun --timeout 900 -- bash tools/gpu_r04_batch.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
TAG=${1:-batch}
mkdir -p gpurun_out/$TAG
run() {  # name env... -- args
  n=$1; shift
  env "$@" timeout -k 10 200 python tools/tile_scaling.py $ARGS > gpurun_out/$TAG/$n.txt 2>&1 || exit $?
  echo "$n $(tail -1 gpurun_out/$TAG/$n.txt)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  ARGS="--counts 8 --ranks-max 1 --frames 24 --inflight 5 --share 25" run s8_b8_f5_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --frames 6 --inflight 5 --share 25 --spp 32" run s8_b32_f5_$r PT_TRI_MIN=3 PT_PASS_BATCH=32
  ARGS="--counts 8 --ranks-max 1 --frames 6 --inflight 3 --share 50 --spp 32" run s8_b32_f3_$r PT_TRI_MIN=3 PT_PASS_BATCH=32
  ARGS="--counts 8 --ranks-max 1 --frames 4 --inflight 2 --share 100 --spp 32" run s8_b32_f2_$r PT_TRI_MIN=3 PT_PASS_BATCH=32
  ARGS="--counts 1 --ranks-max 1 --frames 12 --inflight 3 --share 45" run n1_b8_f3_$r
  ARGS="--counts 1 --ranks-max 1 --frames 4 --inflight 3 --share 45 --spp 32" run n1_b32_f3_$r PT_PASS_BATCH=32
done
