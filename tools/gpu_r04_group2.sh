# Round-4 frame groups at the final kernels (the single-frame instances unchanged, MULTI instances for
# pt_render_frames): parity of render_frames and of the grouped N > 1 pipeline, then rank 0's share per frame
# for G = 1 / 4 / 8 frames per launch at N = 8, 4, 2 and the whole frame at N = 1 (tools/tile_scaling.py).
#   gpurun --timeout 1200 -- bash tools/gpu_r04_group2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
TAG=${1:-group2}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -v -m gpu -k "render_frames or frame_groups or tiled_frames or metric_frame" --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest_gpu.log | head -20; exit $rc; }
run() {  # name env... (ARGS: tile_scaling arguments)
  n=$1; shift
  env "$@" timeout -k 10 200 python tools/tile_scaling.py $ARGS > gpurun_out/$TAG/$n.txt 2>&1 || exit $?
  echo "$n $(tail -1 gpurun_out/$TAG/$n.txt)" | tee -a gpurun_out/$TAG/summary.txt
}
for r in 1 2; do
  ARGS="--counts 8 --ranks-max 1 --frames 24 --inflight 5 --share 25" run s8_g1_f5_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --frames 6 --inflight 3 --share 50 --group 4" run s8_g4_f3_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --frames 4 --inflight 3 --share 50 --group 8" run s8_g8_f3_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --frames 4 --inflight 2 --share 100 --group 8" run s8_g8_f2_$r PT_TRI_MIN=3
  ARGS="--counts 8 --ranks-max 1 --frames 4 --inflight 3 --share 50 --group 8" run s8_g8_f3_tri4_$r
  ARGS="--counts 8 --ranks-max 1 --frames 3 --inflight 3 --share 50 --group 16" run s8_g16_f3_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --frames 24 --inflight 5 --share 25" run s4_g1_f5_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --frames 6 --inflight 3 --share 50 --group 4" run s4_g4_f3_$r PT_TRI_MIN=3
  ARGS="--counts 4 --ranks-max 1 --frames 4 --inflight 3 --share 50 --group 8" run s4_g8_f3_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --frames 24 --inflight 5 --share 25" run s2_g1_f5_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --frames 6 --inflight 3 --share 50 --group 4" run s2_g4_f3_$r PT_TRI_MIN=3
  ARGS="--counts 2 --ranks-max 1 --frames 4 --inflight 3 --share 50 --group 8" run s2_g8_f3_$r PT_TRI_MIN=3
  ARGS="--counts 1 --ranks-max 1 --frames 12 --inflight 3 --share 45" run n1_g1_f3_$r
  ARGS="--counts 1 --ranks-max 1 --frames 6 --inflight 3 --share 45 --group 2" run n1_g2_f3_$r
  ARGS="--counts 1 --ranks-max 1 --frames 3 --inflight 3 --share 45 --group 4" run n1_g4_f3_$r
done
echo done
