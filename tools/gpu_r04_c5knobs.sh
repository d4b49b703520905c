# Round-4: walk knobs on the C5 frame (the textured kernel, 7 waves), alternating with the defaults.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_c5knobs.sh <tag> "VAR=a" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c5knobs}
shift
mkdir -p gpurun_out/$TAG
for r in 1 2; do
for v in "$@"; do
  n=${v//[= ]/_}
  env $v timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/$TAG/b_${n}_$r.json 2> gpurun_out/$TAG/b_${n}_$r.err || exit $?
  echo "$v $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" gpurun_out/$TAG/b_${n}_$r.json)" | tee -a gpurun_out/$TAG/summary.txt
done
done
