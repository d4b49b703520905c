# Round-4 frame groups at N = 1 (LANE_GEN MULTI instances): the whole frame per frame over the 20-frame
# sequence for several group shapes (tools/tile_scaling.py), then the bench line itself with and without
# groups, alternating (the metric, C1 and C2 workloads).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_group6.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
TAG=${1:-group6}
mkdir -p gpurun_out/$TAG
run() {  # name env... (ARGS: tile_scaling arguments)
  n=$1; shift
  env "$@" timeout -k 10 200 python tools/tile_scaling.py $ARGS > gpurun_out/$TAG/$n.txt 2>&1 || exit $?
  echo "$n $(tail -1 gpurun_out/$TAG/$n.txt)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  ARGS="--counts 1 --ranks-max 1 --frames 20 --inflight 3 --share 45" run n1_g1_f3_$r
  ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 2" run n1_g2_f2_$r
  ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 4" run n1_g4_f2_$r
  ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run n1_g8_f2_$r
  ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 3 --share 50 --group 4" run n1_g4_f3_$r
  ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 1 --share 100 --group 4" run n1_g4_f1_$r
done
one() {  # name workload env...
  n=$1; w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/$TAG/b_${n}_$w.json 2> gpurun_out/$TAG/b_${n}_$w.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', 'G', d['config']['frames_per_launch'], 'inflight', d['config']['frames_in_flight'])" gpurun_out/$TAG/b_${n}_$w.json $n $w | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  for w in metric c1 c2; do
    one g1_$r $w PT_BENCH_GROUP=1
    one g4_$r $w PT_BENCH_GROUP=4 PT_BENCH_INFLIGHT=2
  done
done
echo done
