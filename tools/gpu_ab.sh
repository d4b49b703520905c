# GPU step: parity tests, then bench A/B over environment variants (one process per variant).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ab}
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  echo "== $v"
  env $v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench_$(echo $v | tr '= ' '__').json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" gpurun_out/$TAG/bench_$(echo $v | tr '= ' '__').json
done
