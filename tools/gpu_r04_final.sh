# Round-4 final check at the committed tree: the whole -m gpu suite, smoke(), the default bench line (N = 1,
# with its CPU baseline), and the N > 1 bench rehearsal over gloo on one GPU (with and without frame groups).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cut -c1-200 gpurun_out/$TAG/bench.json
bash tools/gpu_multirank_rehearsal.sh $TAG/mr || exit $?
echo done
