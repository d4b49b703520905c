# GPU step: per-rank counters of the tiled share (rank 0 of N = 2, 4, 8), one rocprofv3 --pmc pass per
# counter group, recorded in profiles/traffic.json under "<workload key>/tiled<N>" for bench.py's N > 1
# roofline. Only gpurun_out/ comes back from the GPU box, so the summary is written there too; record
# it here afterwards with
#   python3 tools/traffic_summary.py gpurun_out/share<N> profiles/<round>/share<N> \
#       --workload "<workload key>/tiled<N>" --kernel "pass_kernel_u<8, false, 0, false>" --round <round>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K="pass_kernel_u<8, false, 0, false>"
for N in ${COUNTS:-2 4 8}; do
  D=gpurun_out/share$N
  mkdir -p $D
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $D/pmc_sq -o run -- python3 tools/share_render.py --n $N > $D/sq.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc_fetch -o run -- python3 tools/share_render.py --n $N > $D/fetch.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pmc_write -o run -- python3 tools/share_render.py --n $N > $D/write.log 2>&1 || exit $?
  # the timed mode's kernel at this N: one launch of G = min(8 N, 20) frames of the share (bench.py's frame groups
  # over the driver's 20 steps)
  G=$((8 * N)); [ $G -gt 20 ] && G=20
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $D/pmc_sq_group$G -o run -- python3 tools/share_render.py --n $N --frames 1 --group $G > $D/sq_group.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/share_render.py --n $N > $D/trace.log 2>&1 || exit $?
  cat $D/trace.log
  python3 tools/traffic_summary.py $D $D/summary || exit $?
done
