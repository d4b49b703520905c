# Round-4 step: the hand-over tests, then the metric bench line and the 8-way share (five frames in flight,
# quarter grids, 16 queues; tools/tile_scaling.py) under PT_SPILL / PT_SPILL_GRID variants, two rounds.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_spill.sh <tag> "PT_SPILL=0" "PT_SPILL=16" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-spill}
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "hand_over or metric_frame or c1_" --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest.log | head -20; exit $rc; }
for r in 1 2; do
for v in "$@"; do
  n=${v//[= ]/_}
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/b_${n}_$r.json 2> gpurun_out/$TAG/b_${n}_$r.err || exit $?
  m=$(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['config']['ms_per_frame_latency'])" gpurun_out/$TAG/b_${n}_$r.json)
  env $v GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python tools/tile_scaling.py --counts 8 --ranks-max 1 --frames 24 --inflight 5 --share 25 > gpurun_out/$TAG/t_${n}_$r.txt 2>&1 || exit $?
  s=$(tail -1 gpurun_out/$TAG/t_${n}_$r.txt | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["worst_ms"])')
  echo "$v metric(Mrays/s ms/frame latency) $m share8_ms $s" | tee -a gpurun_out/$TAG/summary.txt
done
done
