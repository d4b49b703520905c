"""Tolerance calibration: the bit-exact oracle against three models of what separates
it from the reference CUDA build (glibc transcendentals for the CUDA intrinsics, nvcc-style FMA
contraction, both), on BASELINE.json's metric frame, a pixel subset, 8 passes. Test infrastructure.

    python tools/tolerance_calibration.py [NPIXELS]
"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import bench, oracle
wl = bench.Workload("metric")
npx = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
sel = np.sort(np.random.default_rng(1).choice(wl.width*wl.height, npx, replace=False)).astype(np.int32)
t = time.time()
a, a8, sa = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 8, pixels=sel, signatures=True)
print("base %.1fs" % (time.time() - t), sa["segments"])
for name, kw in (("libm", dict(math="libm")), ("fma", dict(variant="fma")), ("fma+libm", dict(variant="fma", math="libm"))):
    b, b8, sb = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 8, pixels=sel, signatures=True, **kw)
    d = np.abs(a.astype(np.float64) - b)            # running sum of 8 passes
    dm = d / 8                                       # displayed mean
    flip_unit = sa["signatures"] != sb["signatures"]  # (8, n)
    flip_px = flip_unit.any(axis=0)
    clean = ~flip_px
    rmse = np.sqrt(np.mean((a.astype(np.float64) - b) ** 2)) / a.mean()
    print(f"{name:9s} within1e-3(sum) {np.mean(d.max(1) <= 1e-3):.5f} within1e-3(mean) {np.mean(dm.max(1) <= 1e-3):.5f} "
          f"rmse/mean {rmse:.2e} flipped units {flip_unit.sum()} / {flip_unit.size} ({flip_unit.mean():.2e}) px with a flip {flip_px.mean():.5f} "
          f"max|d| unflipped px {d[clean].max():.3e} (rel {np.max(d[clean] / np.maximum(np.abs(a[clean]), 1e-6)):.2e}) "
          f"px >1e-3 w/o flip {np.sum((d.max(1) > 1e-3) & clean)} u8 diff px {np.mean((a8 != b8).any(1)):.5f} mean shift {(b.mean()-a.mean())/a.mean():+.2e}")
