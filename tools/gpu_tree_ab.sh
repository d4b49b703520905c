# Reference LBVH vs PT_BVH_SAH trees on the GPU (round 6): the bench line A/B (ROUNDS alternating rounds, no
# alternate-tree leg), then per tree one SQ + TCC counter pass over the timed mode's own kernel (the MULTI instance,
# one 8-frame launch) and over the solo launch.
#   gpurun -- bash tools/gpu_tree_ab.sh <tag> [workload]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
TAG=${1:-tree}
W=${2:-metric}
T=gpurun_out/$TAG
mkdir -p $T
for r in $(seq ${ROUNDS:-3}); do
  for v in lbvh sah; do
    timeout -k 10 300 python3 bench.py --workload $W --tree $v --no-alt-tree --no-cpu-baseline ${BENCH_ARGS:-} > $T/cur.json 2>> $T/bench_err.log || exit $?
    cat $T/cur.json >> $T/bench_$v.json
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', r['avg_launch_ms'], 'ms/solo launch')" $T/cur.json $v
  done
done
for v in lbvh sah; do
  # separate passes: FETCH_SIZE takes 3 of the 4 TCC counters a pass may hold
  G="python3 tools/share_render.py --n 1 --frames 2 --workload $W --tree $v"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $T/pmc_sq_group8_$v -o run -- $G --group 8 > $T/pmc_sq_group8_$v.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/pmc_fetch_group8_$v -o run -- $G --group 8 > $T/pmc_fetch_group8_$v.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $T/pmc_tcc_group8_$v -o run -- $G --group 8 > $T/pmc_tcc_group8_$v.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $T/pmc_sq_solo_$v -o run -- $G > $T/pmc_sq_solo_$v.log 2>&1 || exit $?
done
for d in $T/pmc_*_lbvh $T/pmc_*_sah; do echo "== $d"; python3 tools/pmc_summary.py $d; done > $T/pmc_summary.txt 2>&1
cat $T/pmc_summary.txt
