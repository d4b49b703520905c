# Round-4 frame groups with block-aligned frames (no LANE_GEN state): rank 0's share per frame over the
# bench's 20-frame timed sequence, groups against one frame per launch (tools/tile_scaling.py --total).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_group4.sh <tag>     (after tools/gpu_r04_final.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
TAG=${1:-group4}
mkdir -p gpurun_out/$TAG
run() {  # name env... (ARGS: tile_scaling arguments)
  n=$1; shift
  env "$@" timeout -k 10 200 python tools/tile_scaling.py $ARGS > gpurun_out/$TAG/$n.txt 2>&1 || exit $?
  echo "$n $(tail -1 gpurun_out/$TAG/$n.txt)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  ARGS="--counts 8 --ranks-max 1 --frames 20 --inflight 5 --share 25" run s8_g1_f5_t20_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run s8_g8_f2_t20_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --total 40 --inflight 2 --share 100 --group 8" run s8_g8_f2_t40_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run s4_g8_f2_t20_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 4" run s2_g4_f2_t20_$r PT_TRI_MIN=3
  ARGS="--counts 1 --ranks-max 1 --frames 20 --inflight 3 --share 45" run n1_g1_f3_t20_$r
  ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 2" run n1_g2_f2_t20_$r
  ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 3 --share 45 --group 2" run n1_g2_f3_t20_$r
  ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 4" run n1_g4_f2_t20_$r
done
echo done
