# Round-4 profiling step at the final kernel (no parity tests: tools/gpu_r04_check.sh runs those):
#  1. the default bench line (the driver's --steps 20 --warmup 5) and the C1-C5 lines (C4 also --medium-bound);
#  2. rocprofv3 kernel trace + stats of the default command (three frames in flight: the timed mode);
#  3. the same with one frame in flight (PT_BENCH_INFLIGHT=1: a launch's own duration);
#  4. PMC passes, one counter group per run, one frame in flight: FETCH_SIZE, WRITE_SIZE, SQ group;
#  5. PT_UPROF state-machine counters; 6. the PT_DUP phase split (tools/build_dup.sh builds lib_dup*);
#  7. rank 0's share of N = 2, 4, 8 under PMC (tools/gpu_share_pmc.sh).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_profile.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4prof}
mkdir -p gpurun_out/$TAG
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
cut -c1-200 gpurun_out/$TAG/bench.json
for w in c1 c2 c3 c4 c5; do
  timeout -k 10 500 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/$TAG/wl_$w.json 2> gpurun_out/$TAG/wl_$w.err || exit $?
  cut -c1-160 gpurun_out/$TAG/wl_$w.json
done
timeout -k 10 500 python3 bench.py --workload c4 --medium-bound --no-cpu-baseline > gpurun_out/$TAG/wl_c4_mb.json 2> gpurun_out/$TAG/wl_c4_mb.err || exit $?
cut -c1-160 gpurun_out/$TAG/wl_c4_mb.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace_inflight -o run -- $B > gpurun_out/$TAG/trace_inflight.log 2>&1 || exit $?
export PT_BENCH_INFLIGHT=1 PT_BENCH_GROUP=1  # one frame per launch, one at a time: the roofline's solo launch
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/trace.log 2>&1 || exit $?
P="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/pmc_fetch -o run -- $P > gpurun_out/$TAG/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/pmc_write -o run -- $P > gpurun_out/$TAG/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/$TAG/pmc_sq -o run -- $P > gpurun_out/$TAG/pmc_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/$TAG/pmc_sq_group8 -o run -- python3 tools/share_render.py --n 1 --frames 2 --group 8 > gpurun_out/$TAG/pmc_sq_group8.log 2>&1 || exit $?
unset PT_BENCH_INFLIGHT PT_BENCH_GROUP
timeout -k 10 120 python3 tools/uprof.py metric > gpurun_out/$TAG/uprof_metric.json 2> gpurun_out/$TAG/uprof_metric.err || exit $?
if [ -d pathtracerwithcuda_amd/lib_dup1 ]; then
  bash tools/gpu_dup.sh $TAG/dup > gpurun_out/$TAG/dup.log 2>&1 || exit $?
  tail -4 gpurun_out/$TAG/dup.log
fi
bash tools/gpu_share_pmc.sh > gpurun_out/$TAG/share_pmc.log 2>&1 || exit $?
find gpurun_out/$TAG -name "*stats.csv" | head
echo done
