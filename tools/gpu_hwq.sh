# GPU step: frames in flight x grid share x HIP hardware queues (GPU_MAX_HW_QUEUES) for the tiled
# frame (tools/tile_scaling.py, 24 frames per point, rank 0-1 of each N).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hwq2
for cfg in "8 3 50" "8 4 33" "8 5 25" "16 5 25" "16 6 20" "16 8 16" "8 5 20"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 250 python tools/tile_scaling.py --frames 24 --counts 1,2,4,8 --ranks-max 2 --inflight $2 --share $3 > gpurun_out/hwq2/q$1_i$2_s$3.json || exit 1
  echo "q=$1 inflight=$2 share=$3: $(python3 -c "import json,sys; L=[json.loads(l) for l in open(sys.argv[1])]; print(' '.join(f\"N={d['n']} {d['worst_ms']}\" for d in L))" gpurun_out/hwq2/q$1_i$2_s$3.json)"
done
