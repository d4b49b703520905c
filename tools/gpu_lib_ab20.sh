# Parity with an alternative build, then a 20-frame bench A/B against lib/ (two rounds).
#   gpurun -- bash tools/gpu_lib_ab20.sh <tag> <libdir> [env for the alternative, e.g. PT_TRI_MIN=8] ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; ALT=$2; shift 2
mkdir -p gpurun_out/$TAG
if [ -z "$SKIP_TESTS" ]; then
  PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$ALT timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "parity FAILED"; tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
  tail -1 gpurun_out/$TAG/pytest.log
fi
one() {  # name libdir env...
  n=$1; d=$2; shift 2
  env PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$d "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/$n.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" gpurun_out/$TAG/$n.json "$n"
}
for r in 1 2; do
  one base_$r lib
  one alt_$r $ALT
  for e in "$@"; do one alt_${e//[=\/]/_}_$r $ALT $e; done
done
