set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/slp
PT_LIBDIR=/root/repo/pathtracerwithcuda_amd/lib_noslp timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/slp/pytest.log 2>&1 || { tail -30 gpurun_out/slp/pytest.log; exit 1; }
tail -1 gpurun_out/slp/pytest.log
SKIP_TESTS=1 bash tools/gpu_ab.sh slp "PT_UNIFIED=1" "PT_LIBDIR=/root/repo/pathtracerwithcuda_amd/lib_noslp" "PT_UNIFIED=1" "PT_LIBDIR=/root/repo/pathtracerwithcuda_amd/lib_noslp"
