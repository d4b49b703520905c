# Round-4 C4 counters, the exact walk against the medium-bounded one (verdict r03 item 4: nodes per segment,
# SQ_WAIT_ANY and FETCH): the medium-bound GPU tests (HIP frame and instrumented counts against the oracle's
# bounded walk), both bench lines (counts_per_frame from the instrumented kernel), then one C4 frame (32
# launches of 8 passes) under rocprofv3 --pmc per counter group, for each walk.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_c4pmc.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c4pmc}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "medium_bound or instrumented" --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
for m in "" "--medium-bound"; do
  n=exact; [ -n "$m" ] && n=bounded
  timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline $m > gpurun_out/$TAG/bench_$n.json 2> gpurun_out/$TAG/bench_$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['roofline']['counts_per_frame']; print(sys.argv[2], d['value'], 'Mrays/s', 'nodes/segment', round(c['nodes']/c['segments'],2), 'tris/segment', round(c['tris']/c['segments'],2))" gpurun_out/$TAG/bench_$n.json $n | tee -a gpurun_out/$TAG/summary.txt
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/pmc_fetch_$n -o run -- python3 tools/share_render.py --n 1 --frames 1 --workload c4 $m > gpurun_out/$TAG/pmc_fetch_$n.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/$TAG/pmc_sq_$n -o run -- python3 tools/share_render.py --n 1 --frames 1 --workload c4 $m > gpurun_out/$TAG/pmc_sq_$n.log 2>&1 || exit $?
  grep "share 0" gpurun_out/$TAG/pmc_sq_$n.log | tee -a gpurun_out/$TAG/summary.txt
done
echo done
