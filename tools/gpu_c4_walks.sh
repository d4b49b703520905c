# C4 (800k triangles, SSS) and C5 under the alternative walks: default, quantised nodes, wide records.
cd $GRAFT_REPO_ROOT
TAG=${1:-c4walks}
mkdir -p gpurun_out/$TAG
for wl in c4 c5; do
for v in "base" "PT_QNODES=1" "PT_WIDE=1"; do
  f=gpurun_out/$TAG/${wl}_${v%%=*}.json
  env $( [ "$v" = base ] || echo $v ) timeout -k 10 300 python bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['kernel'])" $f "$wl $v"
done
done
