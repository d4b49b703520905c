# SQ counters (one rocprofv3 --pmc pass per variant, one frame in flight) and the PT_UPROF state-machine
# counters of the pass kernel under environment variants:
#   gpurun -- bash tools/gpu_pmc_env.sh <tag> "VAR=a" "VAR=b" ...
# BENCH_ARGS (e.g. "--workload c4") selects the workload; FETCH=1 adds FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
for v in "$@"; do
  n=$(echo $v | tr '= /' '___')
  env PT_BENCH_INFLIGHT=1 $v timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/$TAG/sq_$n -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline $BENCH_ARGS > gpurun_out/$TAG/sq_$n.log 2>&1 || exit $?
  if [ -n "$FETCH" ]; then
    env PT_BENCH_INFLIGHT=1 $v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/fetch_$n -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline $BENCH_ARGS > gpurun_out/$TAG/fetch_$n.log 2>&1 || exit $?
    env PT_BENCH_INFLIGHT=1 $v timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/write_$n -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline $BENCH_ARGS > gpurun_out/$TAG/write_$n.log 2>&1 || exit $?
  fi
  env $v timeout -k 10 120 python3 tools/uprof.py $UPROF_ARGS > gpurun_out/$TAG/uprof_$n.json 2> gpurun_out/$TAG/uprof_$n.err || exit $?
  echo "== $v"
  python3 tools/pmc_summary.py gpurun_out/$TAG > /dev/null
  for d in gpurun_out/$TAG/sq_$n gpurun_out/$TAG/fetch_$n gpurun_out/$TAG/write_$n; do [ -d $d ] && python3 tools/pmc_summary.py $d; done
  cat gpurun_out/$TAG/uprof_$n.json
done
