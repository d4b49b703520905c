# Environment-knob sweep of the tiled frame (tools/tile_scaling.py), one GPU.
#   gpurun --timeout 600 -- bash tools/gpu_env_sweep.sh TAG COUNTS "VAR=a,VAR2=b VAR=c ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-sweep}
mkdir -p gpurun_out/$TAG
for kv in $3; do
  echo "== $kv" >> gpurun_out/$TAG/out.txt
  env ${kv//,/ } timeout -k 10 120 python -u tools/tile_scaling.py --counts $2 --ranks-max 1 >> gpurun_out/$TAG/out.txt 2>&1 || exit $?
done
cat gpurun_out/$TAG/out.txt
