# Round-4 frame-group size at the 8-wave kernel: rank 0's share per frame over the bench's 20-frame sequence,
# G = 4 / 8 / 10 at N = 2 and 4, alternating (tools/tile_scaling.py --total 20, two contexts, whole grid).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_group8.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
TAG=${1:-group8}
mkdir -p gpurun_out/$TAG
run() {  # name env... (ARGS: tile_scaling arguments)
  n=$1; shift
  env "$@" timeout -k 10 200 python tools/tile_scaling.py $ARGS > gpurun_out/$TAG/$n.txt 2>&1 || exit $?
  echo "$n $(tail -1 gpurun_out/$TAG/$n.txt)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  for g in 4 8 10; do
    ARGS="--counts 2 --ranks-max 1 --total 20 --inflight 2 --share 100 --group $g" run s2_g${g}_$r PT_TRI_MIN=3
    ARGS="--counts 4 --ranks-max 1 --total 20 --inflight 2 --share 100 --group $g" run s4_g${g}_$r PT_TRI_MIN=3
  done
done
echo done
