# GPU step: parity tests, then bench A/B over environment variants (one process per variant).
#   gpurun -- bash tools/gpu_ab.sh <tag> "VAR=a VAR2=b" "VAR=c" ...
# STEPS / WARMUP (default 5 / 2) and BENCH_ARGS (e.g. "--workload c4") pass through to bench.py;
# SKIP_TESTS=1 skips the parity suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ab}
shift
mkdir -p gpurun_out/$TAG
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/$TAG/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
for v in "$@"; do
  echo "== $v"
  f=gpurun_out/$TAG/bench_$(echo $v | tr '= /' '___').json
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} --no-cpu-baseline $BENCH_ARGS > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" $f
done
