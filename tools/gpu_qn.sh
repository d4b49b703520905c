set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/qn
PT_QNODES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qn/pytest.log 2>&1 || { tail -20 gpurun_out/qn/pytest.log; exit 1; }
tail -1 gpurun_out/qn/pytest.log
SKIP_TESTS=1 bash tools/gpu_ab.sh qn "PT_QNODES=0" "PT_QNODES=1" "PT_QNODES=1 PT_TRI_MIN=8" "PT_QNODES=1 PT_WALK_STEPS=16" "PT_QNODES=1 PT_MIN_WAVES=6"
