# GPU step: bench A/B over alternative builds, ROUNDS rounds (default 4) of STEPS-frame lines (default 10), the
# builds alternating inside each round; prints Mrays/s, ms/frame and the one-in-flight launch time per line.
#   gpurun -- bash tools/gpu_libab4.sh <tag> <libdir> [<libdir> ...]   (libdir relative to the package)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-libab4}
shift
mkdir -p gpurun_out/$TAG
for r in $(seq 1 ${ROUNDS:-4}); do
for d in "$@"; do
  f=gpurun_out/$TAG/bench_${d}_$r.json
  PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/$d timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline $BENCH_ARGS > $f 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', d['roofline']['avg_launch_ms'], 'ms/launch')" $f $d
done
done
python3 - "$TAG" "$@" <<'PY'
import json, sys, glob, statistics as st
tag, dirs = sys.argv[1], sys.argv[2:]
for d in dirs:
    v = [json.load(open(f)) for f in sorted(glob.glob(f"gpurun_out/{tag}/bench_{d}_[0-9]*.json"))]
    print(f"{d:12s} median {st.median(x['value'] for x in v):9.1f} Mrays/s  launch {st.median(x['roofline']['avg_launch_ms'] for x in v):.4f} ms")
PY
