# GPU step: per-rank counters of the tiled share (rank 0 of N = 2, 4, 8), one rocprofv3 --pmc pass per
# counter group, recorded in profiles/traffic.json under "<workload key>/tiled<N>" for bench.py's N > 1
# roofline (tools/traffic_summary.py). Then the one-GPU frame the same way (key "<workload key>").
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KEY=$(python3 -c "import bench; print(bench.Workload('metric').key)")
K="pass_kernel_u<7, false, 0>"
for N in ${COUNTS:-2 4 8}; do
  D=gpurun_out/share$N
  mkdir -p $D
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $D/pmc_sq -o run -- python3 tools/share_render.py --n $N > $D/sq.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 tools/share_render.py --n $N > $D/fetch.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 tools/share_render.py --n $N > $D/write.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/share_render.py --n $N > $D/trace.log 2>&1 || exit $?
  cat $D/trace.log
  python3 tools/traffic_summary.py $D profiles/r03/share$N --workload "$KEY/tiled$N" --kernel "$K" --round r03 || exit $?
  cp $(find $D/trace -name "*kernel_stats.csv" | head -1) profiles/r03/share$N/kernel_stats.csv
done
