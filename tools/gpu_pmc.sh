# PMC counter passes (one counter group per rocprofv3 run; never combined with tracing domains).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
shift
mkdir -p gpurun_out/$TAG
rocprofv3 -L > gpurun_out/$TAG/counters_list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  env $PMC_ENV timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$TAG/g$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/$TAG/g$i.log 2>&1 || { echo "group $grp failed"; tail -5 gpurun_out/$TAG/g$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/$TAG
