# GPU step: per-rank share cost (rank 0 of N) against frames in flight and grid share, with sixteen
# HIP hardware queues (bench.py's tiled setting).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${HWQ:-16}
mkdir -p gpurun_out/inflight
O=gpurun_out/inflight/sweep.txt
for v in "5 25" "7 16" "9 12" "12 9"; do
  set -- $v
  echo "== inflight $1 share $2 hwq $GPU_MAX_HW_QUEUES" | tee -a $O
  timeout -k 10 240 python tools/tile_scaling.py --counts ${COUNTS:-2,4,8} --ranks-max 1 --frames 24 --inflight $1 --share $2 >> $O 2>&1 || exit $?
  tail -3 $O
done
