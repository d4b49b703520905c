# Round-4 frame groups at N = 1: the default bench line (metric, --steps 20 --warmup 5) with G = 1 (three
# contexts on 45 % grids), and G = 4 / 8 / 10 frames per launch on two contexts over the whole grid, alternating.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_group7.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-group7}
mkdir -p gpurun_out/$TAG
one() {  # name env...
  n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/b_$n.json 2> gpurun_out/$TAG/b_$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', 'G', d['config']['frames_per_launch'], 'inflight', d['config']['frames_in_flight'], 'launch', d['roofline']['avg_launch_ms'])" gpurun_out/$TAG/b_$n.json $n | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2 3; do
  one g1_$r PT_BENCH_GROUP=1
  one g4_$r PT_BENCH_GROUP=4 PT_BENCH_INFLIGHT=2
  one g8_$r PT_BENCH_GROUP=8 PT_BENCH_INFLIGHT=2
  one g10_$r PT_BENCH_GROUP=10 PT_BENCH_INFLIGHT=2
done
echo done
