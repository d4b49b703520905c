# Round-4 frame groups: the block-aligned MULTI refill (lib/) against the LANE_GEN one (lib_gen/, commit
# 261b4ed) on the same box, alternating; rank 0's share per frame over the 20-frame sequence.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_group5.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
TAG=${1:-group5}
mkdir -p gpurun_out/$TAG
run() {  # name libdir env... (ARGS: tile_scaling arguments)
  n=$1; l=$2; shift 2
  env PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$l "$@" timeout -k 10 200 python tools/tile_scaling.py $ARGS > gpurun_out/$TAG/${n}_$l.txt 2>&1 || exit $?
  echo "${n}_$l $(tail -1 gpurun_out/$TAG/${n}_$l.txt)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  for l in lib lib_gen; do
    ARGS="--counts 8 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run s8_g8_f2_t20_$r $l PT_TRI_MIN=3
    ARGS="--counts 4 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run s4_g8_f2_t20_$r $l PT_TRI_MIN=3
    ARGS="--counts 2 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 4" run s2_g4_f2_t20_$r $l PT_TRI_MIN=3
    ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 4" run n1_g4_f2_t20_$r $l
  done
  ARGS="--counts 8 --ranks-max 1 --frames 20 --inflight 5 --share 25" run s8_g1_f5_t20_$r lib PT_TRI_MIN=3
  ARGS="--counts 1 --ranks-max 1 --frames 20 --inflight 3 --share 45" run n1_g1_f3_t20_$r lib
done
echo done
