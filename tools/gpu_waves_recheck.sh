# Occupancy re-check at the final kernel: C4 at 6 vs 7 waves per SIMD, the metric frame at 7 vs 8.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/waves
one() {  # name workload minw steps
  PT_MIN_WAVES=$3 timeout -k 10 300 python bench.py --workload $2 --steps $4 --warmup 2 --no-cpu-baseline > gpurun_out/waves/$1.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['kernel'])" gpurun_out/waves/$1.json $1
}
for r in 1 2; do
  one c4_w6_$r c4 6 3
  one c4_w7_$r c4 7 3
  one m_w7_$r metric 7 20
  one m_w8_$r metric 8 20
done
