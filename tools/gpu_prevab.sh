# GPU step: whole -m gpu suite on the product build, then bench A/B against the previous build kept in
# pathtracerwithcuda_amd/lib_prev (the metric frame at the driver's steps, twice, then C3 / C4 / C5).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-prevab}
mkdir -p gpurun_out/$TAG
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "parity FAILED"; tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
  tail -1 gpurun_out/$TAG/pytest.log
fi
run() {  # <name> <libdir> <bench args...>
  n=$1; L=$2; shift 2
  f=gpurun_out/$TAG/bench_$n.json
  PT_LIBDIR=$L timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" $f $n
}
P=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib
Q=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib_prev
for r in 1 2; do
  run prev_m$r $Q --steps 20 --warmup 5
  run new_m$r $P --steps 20 --warmup 5
done
for w in c3 c4 c5; do
  run prev_$w $Q --steps 3 --warmup 1 --workload $w
  run new_$w $P --steps 3 --warmup 1 --workload $w
done
