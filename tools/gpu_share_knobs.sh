# GPU step: the 8-way share (rank 0, five frames in flight on quarter grids, 16 hardware queues) under
# scheduling-knob variants, two passes over the list (tools/tile_scaling.py).
#   gpurun -- bash tools/gpu_share_knobs.sh <tag> "VAR=a" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
TAG=${1:-share_knobs}
shift
mkdir -p gpurun_out/$TAG
for r in 1 2; do
for v in "$@"; do
  env $v timeout -k 10 120 python tools/tile_scaling.py --counts 8 --ranks-max 1 --frames 24 --inflight 5 --share 25 > gpurun_out/$TAG/run.txt 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/$TAG/run.txt | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["worst_ms"])')" | tee -a gpurun_out/$TAG/summary.txt
done
done
