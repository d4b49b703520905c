# Round-4 final check after the small-launch wave rule: the whole -m gpu suite, smoke(), the C1 and metric bench
# lines, and rank 0's 8-way share counters (its solo launch is now a small one: 7 waves).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_final3.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final3}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/smoke.log
for w in c1 metric; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/$TAG/bench_$w.json 2> gpurun_out/$TAG/bench_$w.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline'].get('kernel_timed'), d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/$TAG/bench_$w.json $w
done
COUNTS=8 bash tools/gpu_share_pmc.sh > gpurun_out/$TAG/share_pmc.log 2>&1 || exit $?
grep "share 0" gpurun_out/$TAG/share_pmc.log
echo done
