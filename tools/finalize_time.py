#!/usr/bin/env python3
"""Rank 0's per-frame 8-bit finalize on one GPU (pt_finalize_u8_image over a 1080p float image), the work the
gather of each rank's own 8-bit rows takes off rank 0.

    python tools/finalize_time.py
"""
import time, torch, sys
sys.path.insert(0, ".")
import bench, pathtracerwithcuda_amd as pt
wl = bench.Workload("metric")
r = pt.Renderer(0); r.upload(wl.scene, wl.cfg); r.setup_frame(wl.width, wl.height)
n = wl.width * wl.height * 3
imgs = [torch.rand(n, device="cuda:0") for _ in range(20)]
imgs8 = [torch.zeros(n, dtype=torch.uint8, device="cuda:0") for _ in range(20)]
for f in range(20): r.finalize_u8_image(wl.cfg, 8, imgs[f], imgs8[f])
r.synchronize(); torch.cuda.synchronize()
t = time.perf_counter()
for rep in range(5):
    for f in range(20): r.finalize_u8_image(wl.cfg, 8, imgs[f], imgs8[f])
r.synchronize(); torch.cuda.synchronize()
print("finalize_u8_image 1080p: %.1f us per frame" % ((time.perf_counter() - t) / 100 * 1e6))
