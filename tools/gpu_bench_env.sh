# Bench A/B over environment settings (one bench process per setting, two rounds).
#   gpurun -- bash tools/gpu_bench_env.sh TAG "VAR=a,VAR2=b VAR=c ..."   ("-" = defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-benv}
mkdir -p gpurun_out/$TAG
for r in 1 2; do
for kv in $2; do
  f=gpurun_out/$TAG/b_${r}_${kv//[,=]/_}.json
  E=""; [ "$kv" != "-" ] && E="${kv//,/ }"
  env $E timeout -k 10 200 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $f "$kv"
done
done
