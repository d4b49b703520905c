# One GPU call for an experimental build <libdir> (package-relative, built with PT_EXTRA_FLAGS): the parity
# suite with it, a 4-round metric A/B against the product build (lib), then one C4 and one C5 line each.
#   gpurun -- bash tools/gpu_variant.sh <tag> <libdir>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-variant}
V=${2:?libdir}
mkdir -p gpurun_out/$TAG
L=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd
PT_LIBDIR=$L/$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_$V.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_$V.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_$V.log
bash tools/gpu_libab4.sh $TAG lib $V || exit $?
for wl in c4 c5; do
  for d in lib $V; do
    PT_LIBDIR=$L/$d timeout -k 10 300 python bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/${wl}_$d.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame')" gpurun_out/$TAG/${wl}_$d.json "$wl $d"
  done
done
