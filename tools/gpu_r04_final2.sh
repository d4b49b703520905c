# Round-4 numbers at the 8-wave kernel: the C1 line at 8 vs 7 waves (PT_PLAIN_WAVES), and rank 0's share per
# frame over the bench's 20-frame sequence with the bench's defaults (tools/tile_scaling.py --total 20).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_final2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final2}
mkdir -p gpurun_out/$TAG
for r in 1 2 3; do
  for w in 8 7; do
    PT_PLAIN_WAVES=$w timeout -k 10 300 python bench.py --workload c1 --no-cpu-baseline > gpurun_out/$TAG/c1_w${w}_$r.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c1 waves', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel'])" gpurun_out/$TAG/c1_w${w}_$r.json $w | tee -a gpurun_out/$TAG/summary.txt
  done
done
export GPU_MAX_HW_QUEUES=16
run() {  # name env... (ARGS: tile_scaling arguments)
  n=$1; shift
  env "$@" timeout -k 10 200 python tools/tile_scaling.py $ARGS > gpurun_out/$TAG/$n.txt 2>&1 || exit $?
  echo "$n $(tail -1 gpurun_out/$TAG/$n.txt)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  ARGS="--counts 8 --ranks-max 1 --frames 20 --inflight 5 --share 25" run s8_g1_f5_t20_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run s8_g8_f2_t20_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run s4_g8_f2_t20_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 4" run s2_g4_f2_t20_$r PT_TRI_MIN=3
  ARGS="--counts 1 --ranks-max 1 --total 20 --inflight 2 --share 100 --group 8" run n1_g8_f2_t20_$r
done
echo done
