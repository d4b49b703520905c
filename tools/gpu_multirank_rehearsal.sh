# Rehearsal of the N > 1 bench path on a one-GPU box: 2, 4 and 8 ranks gathering and 3 reducing over gloo
# (and 2 reducing, 4 and 8 gathering with frame groups),
# every rank on device 0. Each bench line carries config.image_matches_1gpu (rank 0 re-renders the frame
# alone and compares bitwise) and bench.py exits 3 on a mismatch; the saved 8-bit images must also equal the
# 1-GPU image.
#   gpurun --timeout 900 -- bash tools/gpu_multirank_rehearsal.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-mr}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --save-image gpurun_out/$TAG/n1.png > gpurun_out/$TAG/b1.json 2>/dev/null || exit $?
run() {  # name ranks port extra-env...
  m=$1; n=$2; port=$3; shift 3
  env "$@" PT_BENCH_BACKEND=gloo PT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --steps ${S:-5} --warmup 1 --save-image gpurun_out/$TAG/$m.png > gpurun_out/$TAG/$m.json 2> gpurun_out/$TAG/$m.err || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d['config']; pr=c.get('per_rank') or {}; print(sys.argv[2], 'ranks: image_matches_1gpu', c['image_matches_1gpu'], 'frames per launch', c['frames_per_launch'], c['collective']['frame_collective'], d['value'], 'Mrays/s', 'render/collective ms per launch (max over ranks)', pr.get('render_ms_per_launch_max_over_ranks'), pr.get('collective_ms_per_launch_max_over_ranks'))" gpurun_out/$TAG/$m.json $n
  cmp gpurun_out/$TAG/n1.png gpurun_out/$TAG/$m.png || exit 4
}
# b*: one frame per launch (PT_BENCH_GROUP=1); g*: the default frame groups at N > 1 (8 N frames per launch,
# one collective per group; g4, g8, g4s20: the bench's default "gather8", the 8-bit rows per group and the
# float rows after the timed run for the self-check): 5 steps = one launch of 5 frames
run b2 2 29533 PT_FRAME_COLLECTIVE=gather PT_BENCH_GROUP=1
run b3 3 29534 PT_FRAME_COLLECTIVE=reduce PT_BENCH_GROUP=1
run b4 4 29535 PT_FRAME_COLLECTIVE=gather PT_BENCH_GROUP=1
run b8 8 29536 PT_FRAME_COLLECTIVE=gather PT_BENCH_GROUP=1
run g2 2 29537 PT_FRAME_COLLECTIVE=reduce
run g3 3 29538 PT_FRAME_COLLECTIVE=gather
run g4 4 29539 PT_BENCH_GROUP=0
run g8 8 29540 PT_BENCH_GROUP=0
# the driver's 20 steps: with G = 8 N frames per launch, one launch of 20 frames at N = 4 and 8
S=20 run g4s20 4 29541 PT_BENCH_GROUP=0
S=20 run g8s20 8 29542 PT_FRAME_COLLECTIVE=reduce
echo "saved images identical to the 1-GPU image"
