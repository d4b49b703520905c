# GPU step: per-rank share cost with bands in row order, ranked globally, and ranked then dealt over
# the launch's eight regions (renderer.deal_bands), one frame at a time and with frames in flight.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/deal
O=gpurun_out/deal/tile.txt
run() { echo "== $*" | tee -a $O; timeout -k 10 240 python tools/tile_scaling.py --counts 1,8 --ranks-max 2 --frames 6 "$@" >> $O 2>&1 || exit $?; tail -2 $O; }
run
run --order
run --order --deal 8
run --order --deal 8 --band-rows 4
export GPU_MAX_HW_QUEUES=8
run --inflight 5 --share 25
run --inflight 5 --share 25 --order --deal 8
run --inflight 5 --share 25 --order --deal 8 --band-rows 4
run --inflight 3 --share 50 --counts 1
run --inflight 3 --share 50 --counts 1 --order --deal 8
