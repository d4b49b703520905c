# TD/TA busy (vector-memory data return and address units) of the bench kernel under walk variants,
# one frame in flight: default, quantised nodes, one record per step.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/td_ab
for v in "base" "PT_QNODES=1" "PT_WALK_CHAIN=1"; do
  n=${v%%=*}
  env PT_BENCH_INFLIGHT=1 $( [ "$v" = base ] || echo $v ) timeout -s KILL 120 rocprofv3 --pmc TD_TD_BUSY TA_TA_BUSY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU --output-format csv -d gpurun_out/td_ab/$n -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/td_ab/$n.json 2> gpurun_out/td_ab/$n.err || exit $?
  echo "== $v $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['roofline']['avg_launch_ms'], 'ms/launch', d['roofline']['kernel'])" gpurun_out/td_ab/$n.json)"
  python3 tools/pmc_summary.py gpurun_out/td_ab/$n | grep -A6 pass_kernel_u
done
