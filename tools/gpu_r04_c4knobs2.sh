# Round-4: the shading-batch threshold on the medium (C4) and textured (C5) kernels, alternating.
#   gpurun --timeout 1200 -- bash tools/gpu_r04_c4knobs2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c4knobs2}
mkdir -p gpurun_out/$TAG
one() {  # workload env
  w=$1; v=$2
  n=${w}_${v//[= ]/_}_$r
  env $v timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || exit $?
  echo "$w $v $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" gpurun_out/$TAG/$n.json)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  for v in PT_BASE=1 PT_SHADE_MIN=36 PT_SHADE_MIN=40 PT_SHADE_MIN=44 PT_SHADE_MIN=48 "PT_SHADE_MIN=40 PT_WALK_STEPS=12"; do
    one c4 "$v"
  done
  for v in PT_BASE=1 PT_SHADE_MIN=32 PT_SHADE_MIN=36; do
    one c5 "$v"
  done
done
echo done
