# Round-4 step: -m gpu suite; C4 with and without the medium-bounded walk (two rounds each); the multi-rank
# rehearsal (2/3/4/8 ranks on gloo, image_matches_1gpu).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_mb.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-mb}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread --durations=10 > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
for r in 1 2; do
  for mb in "" "--medium-bound"; do
    timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline $mb > gpurun_out/$TAG/c4_${r}${mb}.json 2> gpurun_out/$TAG/c4_${r}${mb}.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4', sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch', d['roofline']['kernel'], 'nodes', d['roofline']['counts_per_frame']['nodes'])" gpurun_out/$TAG/c4_${r}${mb}.json "bound=$mb"
  done
done
bash tools/gpu_multirank_rehearsal.sh $TAG/mr
