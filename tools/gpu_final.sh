# Round-end refresh of every measured number at the current tree, in one GPU call:
#   the -m gpu suite and smoke(); tools/gpu_r03.sh (bench line, timed-mode and one-in-flight traces, PMC passes,
#   PT_UPROF counters, PT_DUP phase split: run tools/build_dup.sh first); tools/gpu_workloads.sh (c2..c5).
#   gpurun --timeout 1200 -- bash tools/gpu_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
bash tools/gpu_r03.sh $TAG || exit $?
bash tools/gpu_workloads.sh $TAG/workloads || exit $?
