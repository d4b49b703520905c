#!/usr/bin/env python3
"""The medium-bounded walk (pt_set_medium_bound, a tolerance mode) against the reference's exact walk, on the
oracle (CPU): whole frames of scenes with participating media, every pixel and every path compared.

For each scene the oracle renders the frame twice — exact (path_tracer_kernel.cu:443-454: every mesh walk starts
with min_t = infinity) and bounded (min_t = free-flight distance * (1 + 2^-10) inside a medium) — with per-path
decision signatures (oracle.render signatures=True: hit primitive and branch per segment). It reports the visit
counts of both walks, the pixels whose float running sum or 8-bit value differ, and the paths whose signature
differs (a pruned walk that changed a hit). DESIGN.md §5 quotes the output (profiles/r05/medium_bound/).

    python tools/medium_bound_study.py [--width 1920 --height 1080 --passes 8 --threads 8] > study.txt
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402  (test infrastructure: this is a study, not the product)

import pathtracerwithcuda_amd as pt  # noqa: E402


def scenes(tmp):
    """(name, scene, cfg, camera kwargs): the reference's subsurface scenes over its own cups and an air medium."""
    import pathlib

    from test_gpu_parity import ASSET_CAMS
    from test_loader import make_root

    root = make_root(pathlib.Path(tmp), assets=True)
    out = []
    for name in ("subsurface_scattering_s", "subsurface_scattering_a"):
        cfg = pt.load_config(str(root / "res" / "configuration" / "config.json"))
        cfg.max_tracer_depth = 8
        sc = pt.load_scene(str(root / "res" / "scene" / f"{name}.json"), root_dir=str(root), config=cfg,
                           background="res\\texture\\lobby", background_format="bmp")
        out.append((name, sc, cfg, ASSET_CAMS[name]))
    # a scattering air over the metric scene: every segment of every path is in a medium (long free flights)
    sc = pt.cornell_scene(pt.torus_knot(350, 100))
    for sig in (0.05, 0.5):
        cfg = pt.configuration(max_tracer_depth=8, air_absorption_coef=(0.02, 0.03, 0.05),
                               air_reduced_scattering_coef=(sig, sig, sig))
        out.append((f"metric_scene_air_sigma_s_{sig}", sc, cfg, dict(pitch=0.08, radius=12.5, center=(0, 1.2, 0))))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--passes", type=int, default=8)
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    import tempfile

    with tempfile.TemporaryDirectory() as tmp:
        for name, sc, cfg, kw in scenes(tmp):
            cam = pt.camera(args.width, args.height, **kw)
            t0 = time.time()
            ex, ex8, se = oracle.render(sc.view, cam, cfg, 1, args.passes, threads=args.threads, signatures=True)
            t1 = time.time()
            bo, bo8, sb = oracle.render(sc.view, cam, cfg, 1, args.passes, threads=args.threads, signatures=True,
                                        medium_bound=True)
            t2 = time.time()
            px = int((~((ex.view(np.uint32) == bo.view(np.uint32)).all(axis=1))).sum())
            px8 = int((~(ex8 == bo8).all(axis=1)).sum())
            paths = int((se["signatures"] != sb["signatures"]).sum())
            d = np.abs(ex.astype(np.float64) - bo).max(axis=1)
            print(f"{name}: {args.width}x{args.height}, {args.passes} passes, depth {cfg.max_tracer_depth}")
            print(f"  exact   segments {se['segments']} nodes {se['nodes']} tris {se['tris']} ({t1 - t0:.1f} s)")
            print(f"  bounded segments {sb['segments']} nodes {sb['nodes']} tris {sb['tris']} ({t2 - t1:.1f} s)"
                  f"  nodes -{100 * (1 - sb['nodes'] / max(se['nodes'], 1)):.1f} %, tris "
                  f"-{100 * (1 - sb['tris'] / max(se['tris'], 1)):.1f} %")
            print(f"  pixels differing {px} (max |d| {d.max():.3g}), 8-bit pixels differing {px8}, paths whose "
                  f"decisions differ {paths} of {se['signatures'].size}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
