# Rehearsal of the N > 1 bench path on a one-GPU box: 2 and 4 ranks (gather), 3 ranks (reduce) over gloo,
# every rank on device 0; the 8-bit images after several frames must equal the 1-GPU image.
mkdir -p gpurun_out/mr
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --save-image gpurun_out/mr/n1.png > gpurun_out/mr/b1.json 2>/dev/null || exit $?
PT_BENCH_BACKEND=gloo PT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --save-image gpurun_out/mr/n2.png > gpurun_out/mr/b2.json 2> gpurun_out/mr/b2.err || exit $?
PT_FRAME_COLLECTIVE=reduce PT_BENCH_BACKEND=gloo PT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 3 --steps 2 --warmup 1 --save-image gpurun_out/mr/n3r.png > gpurun_out/mr/b3.json 2> gpurun_out/mr/b3.err || exit $?
PT_BENCH_BACKEND=gloo PT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 4 --steps 3 --warmup 1 --save-image gpurun_out/mr/n4.png > gpurun_out/mr/b4.json 2> gpurun_out/mr/b4.err || exit $?
cmp gpurun_out/mr/n1.png gpurun_out/mr/n2.png && cmp gpurun_out/mr/n1.png gpurun_out/mr/n3r.png && cmp gpurun_out/mr/n1.png gpurun_out/mr/n4.png && echo "images identical"
