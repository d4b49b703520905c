# GPU step: parity tests with each alternative build (PT_LIBDIR), then bench A/B over the builds.
#   gpurun -- bash tools/gpu_libab.sh <tag> <libdir> [<libdir> ...]   (libdir relative to the package)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-libab}
shift
mkdir -p gpurun_out/$TAG
for d in "$@"; do
  [ -n "$SKIP_TESTS" ] && continue
  PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$d timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_$d.log 2>&1 || { echo "parity FAILED with $d"; tail -30 gpurun_out/$TAG/pytest_$d.log; exit 1; }
  echo "$d: $(tail -1 gpurun_out/$TAG/pytest_$d.log)"
done
for r in 1 2; do
for d in "$@"; do
  f=gpurun_out/$TAG/bench_${d}_$r.json
  PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$d timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" $f $d
done
done
