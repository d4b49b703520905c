# GPU step: parity tests (one pytest process), smoke, short bench. Stops at the first failure.
#   gpurun --timeout 900 -- bash tools/gpu_check.sh [tag] [extra python script]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-check}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest_gpu.log
tail -4 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/smoke.log
if [ -n "$2" ]; then timeout -k 10 300 python $2 > gpurun_out/$TAG/extra.log 2>&1 || exit $?; cat gpurun_out/$TAG/extra.log; fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cat gpurun_out/$TAG/bench.json
