# Tail helper experiment (PT_HELP): parity with lib_help, N=1 bench A/B against lib, and the 8-way tiled share
# one frame at a time and with five frames in flight on quarter grids (tools/tile_scaling.py), both builds.
#   git apply profiles/r03/tail_help/tail_help.patch
#   PT_LIBDIR=$PWD/pathtracerwithcuda_amd/lib_help PT_EXTRA_FLAGS=-DPT_HELP=1 python -m pathtracerwithcuda_amd.build
#   gpurun -- bash tools/gpu_help.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-help}
mkdir -p gpurun_out/$TAG
L=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd
PT_LIBDIR=$L/lib_help timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_help.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_help.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_help.log
ROUNDS=3 bash tools/gpu_libab4.sh $TAG lib lib_help || exit $?
for d in lib lib_help; do
  PT_LIBDIR=$L/$d timeout -k 10 300 python tools/tile_scaling.py --counts 1,8 --frames 3 > gpurun_out/$TAG/tile1_$d.txt 2>&1 || exit $?
  PT_LIBDIR=$L/$d timeout -k 10 300 python tools/tile_scaling.py --counts 8 --frames 5 --inflight 5 --share 25 > gpurun_out/$TAG/tile5_$d.txt 2>&1 || exit $?
  echo "== $d"; tail -4 gpurun_out/$TAG/tile1_$d.txt; tail -3 gpurun_out/$TAG/tile5_$d.txt
done
