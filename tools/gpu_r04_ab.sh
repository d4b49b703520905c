# Round-4 A/B step: the whole -m gpu suite on lib/, then bench lines of lib/ against an alternative build
# (alternating, ROUNDS rounds) for the given workloads, then SQ counters of both on the metric frame.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_ab.sh <tag> <altlibdir> "<workloads>" [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; ALT=$2; WLS=${3:-metric}; ROUNDS=${4:-2}
mkdir -p gpurun_out/$TAG
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
  tail -2 gpurun_out/$TAG/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
fi
one() {  # name libdir workload
  env PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$2 timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline > gpurun_out/$TAG/$1_$3.json 2> gpurun_out/$TAG/$1_$3.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch', d['roofline']['kernel'])" gpurun_out/$TAG/$1_$3.json "$1" "$3"
}
for r in $(seq 1 $ROUNDS); do
  for w in $WLS; do
    one base_$r lib $w
    one alt_$r $ALT $w
  done
done
if [ -n "$PMC" ]; then
  export PT_BENCH_INFLIGHT=1
  for d in lib $ALT; do
    PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$d timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/$TAG/pmc_$d -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/$TAG/pmc_$d.log 2>&1 || exit $?
  done
fi
echo done
