# End-of-batch drain of the tiled share: rank 0's per-frame time over 20 frames (the driver's --steps) vs
# 100 frames, five frames in flight on quarter grids, 16 hardware queues.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/drain
for f in 20 100; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 250 python tools/tile_scaling.py --frames $f --counts 1,8 --ranks-max 1 --inflight 5 --share 25 > gpurun_out/drain/f$f.json || exit 1
  echo "frames=$f: $(tr '\n' ' ' < gpurun_out/drain/f$f.json)"
done
