set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/hwq3
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_multirank.py "tests/test_gpu_parity.py::test_frames_in_flight_equal_one_at_a_time" "tests/test_gpu_parity.py::test_reference_scene_files" > gpurun_out/hwq3/pytest.log 2>&1 || { tail -30 gpurun_out/hwq3/pytest.log; exit 1; }
tail -3 gpurun_out/hwq3/pytest.log
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hwq3/bench_$i.json || exit 1; cut -c1-200 gpurun_out/hwq3/bench_$i.json; done
PT_BENCH_BACKEND=gloo PT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hwq3/bench_n2_rehearsal.json 2> gpurun_out/hwq3/n2.err || { tail -20 gpurun_out/hwq3/n2.err; exit 1; }
cut -c1-300 gpurun_out/hwq3/bench_n2_rehearsal.json
