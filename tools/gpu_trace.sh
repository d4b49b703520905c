# GPU step: kernel-trace summary (rocprofv3 --kernel-trace --stats) of a short bench, per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-trace}
shift
mkdir -p gpurun_out/$TAG
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== $v"
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/v$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/v$i.log 2>&1 || { tail -5 gpurun_out/$TAG/v$i.log; exit 1; }
  python3 - gpurun_out/$TAG/v$i/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):5.1f}")
PY
done
