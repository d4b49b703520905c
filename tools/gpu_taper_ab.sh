# Tapered work chunks A/B (round 6, lost; the kernel change is profiles/r06/taper/tapered_chunks.patch: apply it with
# `git apply` and rebuild first): the bench line and its solo launch at N = 1, then rank 0's 8-way share over the
# driver's 20 frames (one launch of 20 frames, tools/tile_scaling.py). PT_CHUNK_TAIL 64 = off.
#   gpurun -- bash tools/gpu_taper_ab.sh <tag> [variants: "tail:rounds ..."]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
TAG=${1:-taper}
V=${2:-"64:2 16:2 8:2 16:4"}
T=gpurun_out/$TAG
mkdir -p $T
for r in $(seq ${ROUNDS:-2}); do
  for v in $V; do
    PT_CHUNK_TAIL=${v%%:*} PT_TAPER_ROUNDS=${v##*:} timeout -k 10 300 python3 bench.py --no-alt-tree --no-cpu-baseline > $T/cur.json 2>> $T/err.log || exit $?
    cat $T/cur.json >> $T/bench_$v.json
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('bench', sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', r['avg_launch_ms'], 'ms/solo launch', d['config']['ms_per_frame_latency'], 'ms latency')" $T/cur.json $v
  done
done
for r in $(seq ${ROUNDS:-2}); do
  for v in $V; do
    PT_CHUNK_TAIL=${v%%:*} PT_TAPER_ROUNDS=${v##*:} PT_TRI_MIN=3 GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 tools/tile_scaling.py --counts 8 --ranks-max 2 --group 64 --inflight 2 --total 20 > $T/tile_$v.json 2>> $T/err.log || exit $?
    echo "tile8 $v $(tr -d '\n' < $T/tile_$v.json | head -c 600)"
  done
done
