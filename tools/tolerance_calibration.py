"""Tolerance calibration: the bit-exact oracle against models of what separates it from
the reference CUDA build, on a BASELINE.json frame (pixel subset, 8 passes). Test infrastructure.

Models: glibc transcendentals for the intrinsics ("libm"); the contraction sites unfused ("plain": an nvcc
--fmad=false build); gcc's own contraction of everything (-ffp-contract=fast, "fma"); combinations;
the documented maximum errors of the CUDA intrinsics the reference calls (__sinf/__cosf/__tanf/__expf/
__logf/__powf and rsqrtf, oracle_math.h OR_MATH_CUDA: the direction keyed by the function's input;
"cuda_site": keyed by (pass, pixel, depth, call)), with and without contraction.

    python tools/tolerance_calibration.py [WORKLOAD] [NPIXELS (0: whole frame)] [SEED]
"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import bench, oracle

MODELS = (("libm", dict(math="libm")), ("plain", dict(arith="plain")), ("plain+libm", dict(arith="plain", math="libm")),
          ("fma", dict(variant="fma")), ("fma+libm", dict(variant="fma", math="libm")),
          ("cuda", dict(math="cuda")), ("cuda_site", dict(math="cuda_site")), ("plain+cuda", dict(arith="plain", math="cuda")),
          ("plain+cuda_site", dict(arith="plain", math="cuda_site")), ("fma+cuda", dict(variant="fma", math="cuda")))


def compare(a, a8, sa, b, b8, sb, passes=8):
    """The statistics of the stated tolerance (tests/test_oracle.py): per pixel of the running
    sum, split by whether the path topology changed (a flip: another hit primitive, branch or sky face in
    some pass) — flips are a resample of the path, unflipped pixels differ by rounding only."""
    a64 = a.astype(np.float64)
    diff = b.astype(np.float64) - a64
    d = np.abs(diff)
    flip_unit = sa["signatures"] != sb["signatures"]  # (passes, n)
    flip_px = flip_unit.any(axis=0)
    clean = ~flip_px
    mean = a64.mean()
    fd = diff[flip_px]
    return {
        "within1e-3": float(np.mean(d.max(1) <= 1e-3)),
        "px_with_flip": float(flip_px.mean()),
        "px_over_1e-3_without_flip": int(np.sum((d.max(1) > 1e-3) & clean)),
        "rmse_over_mean": float(np.sqrt(np.mean(diff ** 2)) / mean),
        "mean_shift": float(diff.mean() / mean),
        "unflipped_rmse_over_mean": float(np.sqrt(np.mean(diff[clean] ** 2)) / mean) if clean.any() else 0.0,
        "unflipped_mean_shift": float(diff[clean].sum() / d.shape[0] / d.shape[1] / mean) if clean.any() else 0.0,
        "flipped_sum_z": float(abs(fd.sum()) / np.sqrt((fd ** 2).sum())) if fd.size and (fd ** 2).sum() > 0 else 0.0,
        "max_rel_unflipped": float(np.max(d[clean] / np.maximum(np.abs(a[clean]), 1e-6))) if clean.any() else 0.0,
        "identical_px": float(np.mean(d.max(1) == 0)),
        "u8_diff_px": float(np.mean((a8 != b8).any(1))),
        "finite": bool(np.isfinite(b).all()),
    }


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "metric"
    npx = int(sys.argv[2]) if len(sys.argv) > 2 else 20000  # 0: the whole frame
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    wl = bench.Workload(name)
    sel = (np.sort(np.random.default_rng(seed).choice(wl.width * wl.height, npx, replace=False)).astype(np.int32)
           if npx else None)
    t = time.time()
    a, a8, sa = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 8, pixels=sel, signatures=True)
    print(f"{name}: {npx or wl.width * wl.height} px (seed {seed}) x 8 passes, base {time.time() - t:.1f}s, "
          f"{sa['segments']} segments")
    for m, kw in MODELS:
        b, b8, sb = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 8, pixels=sel, signatures=True, **kw)
        r = compare(a, a8, sa, b, b8, sb)
        print(f"{m:14s} " + " ".join(f"{k} {v:.5g}" if isinstance(v, float) else f"{k} {v}" for k, v in r.items()))


if __name__ == "__main__":
    main()
