# Round-4 GPU step: the whole -m gpu suite (whole-frame parity), smoke, the default bench line and C1's line.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_check.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4check}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread --durations=15 > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest_gpu.log
tail -4 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cut -c1-200 gpurun_out/$TAG/bench.json
timeout -k 10 300 python bench.py --workload c1 > gpurun_out/$TAG/bench_c1.json 2> gpurun_out/$TAG/bench_c1.err || exit $?
cut -c1-200 gpurun_out/$TAG/bench_c1.json
