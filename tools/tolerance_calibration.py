"""Tolerance calibration: the bit-exact oracle against models of what separates it from
the reference CUDA build, on a BASELINE.json frame (pixel subset, 8 passes). Test infrastructure.

Models: glibc transcendentals for the intrinsics ("libm"); nvcc-style FMA contraction ("fma"); both;
the documented maximum errors of the CUDA intrinsics the reference calls (__sinf/__cosf/__tanf/__expf/
__logf/__powf and rsqrtf, oracle_math.h OR_MATH_CUDA: the direction keyed by the function's input;
"cuda_site": keyed by (pass, pixel, depth, call)), with and without contraction.

    python tools/tolerance_calibration.py [WORKLOAD] [NPIXELS]
"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import bench, oracle

MODELS = (("libm", dict(math="libm")), ("fma", dict(variant="fma")), ("fma+libm", dict(variant="fma", math="libm")),
          ("cuda", dict(math="cuda")), ("cuda_site", dict(math="cuda_site")), ("fma+cuda", dict(variant="fma", math="cuda")),
          ("fma+cuda_site", dict(variant="fma", math="cuda_site")))


def compare(a, a8, sa, b, b8, sb, passes=8):
    d = np.abs(a.astype(np.float64) - b)            # running sum of the passes
    flip_unit = sa["signatures"] != sb["signatures"]  # (passes, n)
    flip_px = flip_unit.any(axis=0)
    clean = ~flip_px
    return {
        "within1e-3": float(np.mean(d.max(1) <= 1e-3)),
        "rmse_over_mean": float(np.sqrt(np.mean((a.astype(np.float64) - b) ** 2)) / a.mean()),
        "mean_shift": float((b.mean() - a.mean()) / a.mean()),
        "flipped_units": float(flip_unit.mean()),
        "px_with_flip": float(flip_px.mean()),
        "px_over_1e-3_without_flip": int(np.sum((d.max(1) > 1e-3) & clean)),
        "max_rel_unflipped": float(np.max(d[clean] / np.maximum(np.abs(a[clean]), 1e-6))) if clean.any() else 0.0,
        "u8_diff_px": float(np.mean((a8 != b8).any(1))),
        "finite": bool(np.isfinite(b).all()),
    }


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "metric"
    npx = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    wl = bench.Workload(name)
    sel = np.sort(np.random.default_rng(1).choice(wl.width * wl.height, npx, replace=False)).astype(np.int32)
    t = time.time()
    a, a8, sa = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 8, pixels=sel, signatures=True)
    print(f"{name}: {npx} px x 8 passes, base {time.time() - t:.1f}s, {sa['segments']} segments")
    for m, kw in MODELS:
        b, b8, sb = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 8, pixels=sel, signatures=True, **kw)
        r = compare(a, a8, sa, b, b8, sb)
        print(f"{m:14s} " + " ".join(f"{k} {v:.5g}" if isinstance(v, float) else f"{k} {v}" for k, v in r.items()))


if __name__ == "__main__":
    main()
