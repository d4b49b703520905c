# Deferred leaves (PT_DEFER build in lib_defer): parity with that build, then bench A/B against lib/ and a
# PT_TRI_MIN sweep of the deferred build.   gpurun -- bash tools/gpu_defer_ab.sh <tag> [tri_min ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-defer}
shift
mkdir -p gpurun_out/$TAG
D=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib_defer
if [ -z "$SKIP_TESTS" ]; then
  PT_LIBDIR=$D timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_defer.log 2>&1 || { echo "parity FAILED"; tail -40 gpurun_out/$TAG/pytest_defer.log; exit 1; }
  tail -1 gpurun_out/$TAG/pytest_defer.log
fi
one() {  # name libdir tri_min
  f=gpurun_out/$TAG/bench_$1.json
  PT_LIBDIR=$2 PT_TRI_MIN=$3 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" $f $1
}
for r in 1 2; do
  one base_$r $GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib 6
  for t in "${@:-16}"; do one defer_t${t}_$r $D $t; done
done
