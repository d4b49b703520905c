# Round-4: contexts for the multi-launch frames (C3, C4): three on half grids (C4) / 45 % (C3), the default,
# against two on the whole grid, alternating.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_ctx2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ctx2}
mkdir -p gpurun_out/$TAG
one() {  # name workload env...
  n=$1; w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', 'inflight', d['config']['frames_in_flight'], 'share', d['config']['grid_share_pct'])" gpurun_out/$TAG/$n.json $n | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  for w in c3 c4; do
    one ${w}_default_$r $w PT_BASE=1
    one ${w}_two_$r $w PT_BENCH_INFLIGHT=2
  done
done
echo done
