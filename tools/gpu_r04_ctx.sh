# Round-4: frame groups on two contexts (whole grid) or three (half grids) at N = 1, over the driver's 20 timed
# frames and over 40 and 60, alternating.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_ctx.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ctx}
mkdir -p gpurun_out/$TAG
one() {  # name steps env...
  n=$1; k=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --steps $k > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', 'inflight', d['config']['frames_in_flight'], 'share', d['config']['grid_share_pct'])" gpurun_out/$TAG/$n.json $n | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  for k in 20 40 60; do
    one c2_s${k}_$r $k PT_BENCH_INFLIGHT=2
    one c3_s${k}_$r $k PT_BENCH_INFLIGHT=3
  done
done
echo done
