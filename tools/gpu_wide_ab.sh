# Wide-walk A/B on one GPU: parity tests, then bench.py alternating PT_WIDE=1 / PT_WIDE=0 (two rounds),
# then the PT_UPROF state-machine counters of both walks (walk steps per segment, lanes per step).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-wide}
SKIP_TESTS=${SKIP_TESTS:-0}
mkdir -p gpurun_out/$TAG
if [ "$SKIP_TESTS" = 0 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
  echo "pytest exit $rc" >> gpurun_out/$TAG/pytest_gpu.log
  tail -4 gpurun_out/$TAG/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
for round in 1 2; do
  for w in 1 0; do
    PT_WIDE=$w timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/$TAG/b${round}_w$w.json 2> gpurun_out/$TAG/b${round}_w$w.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/$TAG/b${round}_w$w.json')); print('round $round PT_WIDE=$w', d['value'], d['ms_per_step'], d['config']['ms_per_frame_latency'], d['roofline']['avg_launch_ms'])"
  done
done
for w in 1 0; do
  PT_WIDE=$w timeout -k 10 300 python tools/uprof.py > gpurun_out/$TAG/uprof_w$w.json 2> gpurun_out/$TAG/uprof_w$w.err || exit $?
  cat gpurun_out/$TAG/uprof_w$w.json
done
echo done
