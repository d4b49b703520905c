# Round-4 register step: the hit point computed where it is used and the clamp bound at use (pt_path.h,
# pt_kernels.hip) bring the bench kernel to 64 VGPRs without spills (8 waves/SIMD possible) and the medium
# kernel to 72 (7 waves); the medium-bound state only in PT_FEAT_MBOUND instances. Whole -m gpu suite, the
# metric parity tests at 8 waves, then bench lines against the previous commit (lib_prev), alternating.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_waves.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-waves}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
PT_MIN_WAVES=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "metric_frame or c3 or variants or edge" --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_w8.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_w8.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_w8.log | head -20; exit $rc; }
one() {  # name libdir workload env...
  n=$1; l=$2; w=$3; shift 3
  env PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$l "$@" timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch', d['roofline'].get('kernel_timed'))" gpurun_out/$TAG/$n.json $n | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  one new_metric_$r lib metric
  one prev_metric_$r lib_prev metric
  one new_metric_w8_g1_$r lib metric PT_MIN_WAVES=8 PT_BENCH_GROUP=1
  one new_metric_g1_$r lib metric PT_BENCH_GROUP=1
  one prev_metric_g1_$r lib_prev metric PT_BENCH_GROUP=1
  one new_c4_$r lib c4
  one new_c4_w6_$r lib c4 PT_MEDIUM_WAVES=6
  one prev_c4_$r lib_prev c4
  one new_c3_$r lib c3
  one new_c3_w8_$r lib c3 PT_MIN_WAVES=8
  one prev_c3_$r lib_prev c3
  one new_c5_$r lib c5
  one prev_c5_$r lib_prev c5
done
echo done
