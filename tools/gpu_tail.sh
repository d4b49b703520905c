# Tail-threshold sweep of pass_kernel_u on the tiled frame (tools/tile_scaling.py), one GPU.
#   gpurun --timeout 600 -- bash tools/gpu_tail.sh TAG "S:W S:W ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-tail}
mkdir -p gpurun_out/$TAG
for sw in $2; do
  s=${sw%%:*}; w=${sw##*:}
  echo "== tail shade_min $s walk_min $w" >> gpurun_out/$TAG/out.txt
  PT_TAIL_SHADE_MIN=$s PT_TAIL_WALK_MIN=$w timeout -k 10 120 python -u tools/tile_scaling.py --counts ${3:-1,8,128} --ranks-max 1 >> gpurun_out/$TAG/out.txt 2>&1 || exit $?
done
cat gpurun_out/$TAG/out.txt
