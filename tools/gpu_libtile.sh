# Parity tests + tiled-frame timings (tools/tile_scaling.py) for alternative builds (PT_LIBDIR), one GPU.
#   gpurun -- bash tools/gpu_libtile.sh <tag> <counts> <libdir> [<libdir> ...]   (libdir relative to the package)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-libtile}; COUNTS=$2
shift 2
mkdir -p gpurun_out/$TAG
for d in "$@"; do
  L=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$d
  PT_LIBDIR=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_$d.log 2>&1 || { echo "parity FAILED with $d"; tail -30 gpurun_out/$TAG/pytest_$d.log; exit 1; }
  echo "$d: $(tail -1 gpurun_out/$TAG/pytest_$d.log)"
  for f in 1 3; do
    echo "== $d inflight $f" >> gpurun_out/$TAG/out.txt
    PT_LIBDIR=$L timeout -k 10 120 python -u tools/tile_scaling.py --counts $COUNTS --ranks-max 1 --frames 6 --inflight $f >> gpurun_out/$TAG/out.txt 2>&1 || exit $?
  done
done
cat gpurun_out/$TAG/out.txt
