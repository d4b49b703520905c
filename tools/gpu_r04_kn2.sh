set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/kn2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "reference_abi" --timeout 200 --timeout-method thread > gpurun_out/kn2/pytest.log 2>&1 || { tail -30 gpurun_out/kn2/pytest.log; exit 1; }
tail -1 gpurun_out/kn2/pytest.log
ABI=1 bash tools/gpu_r04_knobs.sh kn2 "PT_TRI_MIN=6" "PT_TRI_MIN=4" "PT_TRI_MIN=3" "PT_TRI_MIN=5" "PT_TRI_MIN=4 PT_WALK_MIN=10"
