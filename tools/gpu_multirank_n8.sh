# Rehearsal of the 8-rank bench path on a one-GPU box (gloo, every rank on device 0, five frames in
# flight per rank): the 8-bit image must equal the 1-GPU image. RCCL itself runs only on the driver's node.
mkdir -p gpurun_out/mr8
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --save-image gpurun_out/mr8/n1.png > gpurun_out/mr8/b1.json 2>/dev/null || exit $?
PT_BENCH_BACKEND=gloo PT_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --steps 3 --warmup 1 --save-image gpurun_out/mr8/n8.png > gpurun_out/mr8/b8.json 2> gpurun_out/mr8/b8.err || exit $?
cmp gpurun_out/mr8/n1.png gpurun_out/mr8/n8.png && echo "8-rank image identical to 1-GPU image"
