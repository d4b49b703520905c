# Parity with the current library, then bench A/B of one environment switch: gpurun -- bash tools/gpu_env_ab2.sh <tag> VAR=a VAR=b ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "parity FAILED"; tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
  tail -1 gpurun_out/$TAG/pytest.log
fi
for r in 1 2; do for v in "$@"; do
  f=gpurun_out/$TAG/bench_${v//[=\/]/_}_$r.json
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" $f "$v"
done; done
