# One GPU call for an iteration: the parity suite on the product build (lib), a ROUNDS x STEPS bench A/B of
# lib against lib_prev (the previous build), then optional environment variants of the product build.
#   gpurun -- bash tools/gpu_step.sh <tag> ["VAR=a" ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-step}
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/gpu_libab4.sh $TAG lib_prev lib || exit $?
if [ $# -gt 0 ]; then SKIP_TESTS=1 STEPS=10 WARMUP=3 bash tools/gpu_ab.sh $TAG/env "$@" || exit $?; fi
