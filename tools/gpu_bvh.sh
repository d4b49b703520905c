# Row f1 on the GPU: the device BVH tests, then the build timings with the second half on the host
# (round 1) and on the device.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-bvh}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/$TAG/pytest_gpu.log
tail -5 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
PT_BVH_DEVICE_FINISH=0 timeout -k 10 300 python tools/bvh_timing.py > gpurun_out/$TAG/bvh_timing_hostfinish.jsonl || exit $?
timeout -k 10 300 python tools/bvh_timing.py > gpurun_out/$TAG/bvh_timing_devicefinish.jsonl || exit $?
cat gpurun_out/$TAG/bvh_timing_*.jsonl
