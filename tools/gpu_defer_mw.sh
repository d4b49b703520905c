# Deferred leaves vs base at 6 and 7 waves per SIMD (PT_MIN_WAVES), bench frame.
cd $GRAFT_REPO_ROOT
TAG=${1:-defer_mw}
mkdir -p gpurun_out/$TAG
one() {  # name libdir minw tri_min
  f=gpurun_out/$TAG/bench_$1.json
  PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$2 PT_MIN_WAVES=$3 PT_TRI_MIN=$4 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch', d['roofline']['kernel'])" $f $1
}
for r in 1 2; do
  one base_w7_$r lib 7 6
  one base_w6_$r lib 6 6
  one defer_w7_$r lib_defer 7 16
  one defer_w6_$r lib_defer 6 16
done
