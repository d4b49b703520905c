# The BASELINE.json multi-GPU configurations rehearsed over gloo on the one-GPU box: C4 tiled across 4 ranks (its
# default gather) and C5 across 8 with the float reduce ("RCCL accum"), one timed frame each, every rank on device 0.
# Each line carries config.image_matches_1gpu (rank 0 re-renders the frame alone and compares bitwise).
#   gpurun --timeout 900 -- bash tools/gpu_heavy_rehearsal.sh [tag]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
TAG=${1:-heavy}
mkdir -p gpurun_out/$TAG
run() {  # name workload ranks port extra-args...
  m=$1; w=$2; n=$3; port=$4; shift 4
  PT_BENCH_BACKEND=gloo PT_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --workload $w --steps 1 --warmup 0 "$@" > gpurun_out/$TAG/$m.json 2> gpurun_out/$TAG/$m.err || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; pr=c.get('per_rank') or {}; print(sys.argv[2], c['workload'], d['n_gpus'], 'ranks: image_matches_1gpu', c['image_matches_1gpu'], c['collective']['frame_collective'], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', 'render/collective ms (max over ranks)', pr.get('render_ms_per_launch_max_over_ranks'), pr.get('collective_ms_per_launch_max_over_ranks'))" gpurun_out/$TAG/$m.json $m
}
run c4n4 c4 4 29551
run c5n8 c5 8 29552 --collective reduce
