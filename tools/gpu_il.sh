# GPU step (round 3, kept for the record: inline leaves are now the product): a variant build in ILDIR: whole -m gpu suite on it, then bench
# A/B against the product build on the metric frame (driver's steps) and on C4 / C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-il}
mkdir -p gpurun_out/$TAG
IL=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/${ILDIR:-lib_il}
if [ -z "$SKIP_TESTS" ]; then
  PT_LIBDIR=$IL timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_il.log 2>&1 || { echo "parity FAILED"; tail -30 gpurun_out/$TAG/pytest_il.log; exit 1; }
  tail -1 gpurun_out/$TAG/pytest_il.log
fi
run() {  # <name> <libdir> <bench args...>
  n=$1; L=$2; shift 2
  f=gpurun_out/$TAG/bench_$n.json
  PT_LIBDIR=$L timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" $f $n
}
P=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib
for r in 1 2; do
  run base_m$r $P --steps 20 --warmup 5
  run il_m$r $IL --steps 20 --warmup 5
done
run base_c4 $P --steps 3 --warmup 1 --workload c4
run il_c4 $IL --steps 3 --warmup 1 --workload c4
run base_c5 $P --steps 3 --warmup 1 --workload c5
run il_c5 $IL --steps 3 --warmup 1 --workload c5
