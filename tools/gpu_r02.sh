# Round-2 GPU step: parity tests, smoke, the default bench line, then rocprofv3 summaries of the bench
# command with ONE frame in flight (PT_BENCH_INFLIGHT=1: a launch's duration is not stretched by an
# overlapping frame): kernel trace + stats, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ group).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
SKIP_TESTS=${SKIP_TESTS:-0}
mkdir -p gpurun_out/$TAG
if [ "$SKIP_TESTS" = 0 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
  echo "pytest exit $rc" >> gpurun_out/$TAG/pytest_gpu.log
  tail -4 gpurun_out/$TAG/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc  # a failure may be a GPU fault: nothing more on the GPU in this call
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
  tail -1 gpurun_out/$TAG/smoke.log
fi
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cat gpurun_out/$TAG/bench.json
export PT_BENCH_INFLIGHT=1
P="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/pmc_fetch -o run -- $P > gpurun_out/$TAG/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/pmc_write -o run -- $P > gpurun_out/$TAG/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/$TAG/pmc_sq -o run -- $P > gpurun_out/$TAG/pmc_sq.log 2>&1 || exit $?
find gpurun_out/$TAG -name "*stats.csv"
echo done
