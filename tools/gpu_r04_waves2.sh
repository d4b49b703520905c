# Round-4 register step, second form: 8 waves for scenes without textures or media (single-frame and MULTI
# instances), the hit point recomputed at use only there, media at 6 waves. Whole -m gpu suite, then bench
# lines against the previous commit (lib_prev), alternating, three rounds.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_waves2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-waves2}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
one() {  # name libdir workload env...
  n=$1; l=$2; w=$3; shift 3
  env PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$l "$@" timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch', d['roofline'].get('kernel_timed'))" gpurun_out/$TAG/$n.json $n | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2 3; do
  one new_metric_$r lib metric
  one prev_metric_$r lib_prev metric
  one new_metric_g1_$r lib metric PT_BENCH_GROUP=1
  one prev_metric_g1_$r lib_prev metric PT_BENCH_GROUP=1
done
for r in 1 2; do
  one new_c2_$r lib c2
  one prev_c2_$r lib_prev c2
  one new_c3_$r lib c3
  one prev_c3_$r lib_prev c3
  one new_c4_$r lib c4
  one prev_c4_$r lib_prev c4
  one new_c5_$r lib c5
  one prev_c5_$r lib_prev c5
done
echo done
