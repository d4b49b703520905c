# A/B of environment knobs on the bench (one GPU): each argument is an env assignment list ("-" = none),
# run in two alternating rounds; prints value, ms/frame, latency, solo launch ms per run.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for round in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    envs=""; [ "$cfg" != "-" ] && envs="$cfg"
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup ${WARMUP:-3} > gpurun_out/$TAG/b${round}_$i.json 2> gpurun_out/$TAG/b${round}_$i.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/$TAG/b${round}_$i.json')); print('round $round [$cfg]', d['value'], d['ms_per_step'], d['config']['ms_per_frame_latency'], d['roofline']['avg_launch_ms'])"
  done
done
