# Round-3 profiling step (no parity tests: run tools/gpu_check.sh for those):
#  1. the default bench line (the driver's --steps 20 --warmup 5);
#  2. rocprofv3 kernel trace + stats of that same command (three frames in flight: the timed mode);
#  3. the same with one frame in flight (PT_BENCH_INFLIGHT=1: a launch's own duration);
#  4. PMC passes, one counter group per run, one frame in flight: FETCH_SIZE, WRITE_SIZE, SQ group;
#  5. PT_UPROF state-machine counters; 6. the PT_DUP phase split (tools/build_dup.sh builds lib_dup*).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out/$TAG
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 $B > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cut -c1-160 gpurun_out/$TAG/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace_inflight -o run -- $B > gpurun_out/$TAG/trace_inflight.log 2>&1 || exit $?
export PT_BENCH_INFLIGHT=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/trace.log 2>&1 || exit $?
P="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/pmc_fetch -o run -- $P > gpurun_out/$TAG/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/pmc_write -o run -- $P > gpurun_out/$TAG/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/$TAG/pmc_sq -o run -- $P > gpurun_out/$TAG/pmc_sq.log 2>&1 || exit $?
unset PT_BENCH_INFLIGHT
timeout -k 10 120 python3 tools/uprof.py metric > gpurun_out/$TAG/uprof_metric.json 2> gpurun_out/$TAG/uprof_metric.err || exit $?
if [ -d pathtracerwithcuda_amd/lib_dup1 ]; then
  bash tools/gpu_dup.sh $TAG/dup > gpurun_out/$TAG/dup.log 2>&1 || exit $?
  tail -4 gpurun_out/$TAG/dup.log
fi
find gpurun_out/$TAG -name "*stats.csv" | head
echo done
