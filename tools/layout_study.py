#!/usr/bin/env python3
"""STUDY TOOL: dependent record loads per mesh walk under two node-record layouts (tools/layout_study.c),
replayed on the rays of the bench frame. CPU only; test infrastructure (uses the oracle)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bench  # noqa: E402  (scene constants)
import oracle  # noqa: E402
import pathtracerwithcuda_amd as pt  # noqa: E402

NAMES = ["calls", "visits", "chain2_steps", "children_steps_reload", "children_steps_kept", "tri_tests"]


def main():
    sample = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    so = "/tmp/liblayout.so"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                    "-shared", os.path.join(ROOT, "tools", "layout_study.c"), "-o", so, "-lm"], check=True)
    oracle.build()
    oracle.VARIANTS[""] = so
    L = oracle.lib()
    L.layout_stats.argtypes = [C.c_void_p, C.c_void_p]
    scene = pt.cornell_scene(pt.torus_knot(*bench.KNOT))
    cfg = pt.configuration(max_tracer_depth=bench.DEPTH)
    cam = pt.camera(bench.WIDTH, bench.HEIGHT, **bench.CAMERA)
    pix = np.sort(np.random.default_rng(1).choice(bench.WIDTH * bench.HEIGHT, size=sample, replace=False)).astype(np.int32)
    t0 = time.time()
    oracle.render(scene.view, cam, cfg, 1, passes, pixels=pix, with_u8=False)
    tot = (C.c_ulonglong * len(NAMES))()
    per = (C.c_ulonglong * (16 * len(NAMES)))()
    L.layout_stats(tot, per)
    print(f"{sample} px x {passes} passes, {time.time() - t0:.1f} s")
    rows = [("all", list(tot))] + [(f"mesh {m}", list(per)[m * len(NAMES):(m + 1) * len(NAMES)]) for m in range(16)]
    for name, v in rows:
        if not v[0]:
            continue
        d = dict(zip(NAMES, v))
        c = d["calls"]
        print(f"{name}: walks {c}, per walk: visits {d['visits'] / c:.2f}, chain2 {d['chain2_steps'] / c:.2f}, "
              f"children (reload after a leaf) {d['children_steps_reload'] / c:.2f}, (kept) {d['children_steps_kept'] / c:.2f}, "
              f"triangle tests {d['tri_tests'] / c:.2f}")


if __name__ == "__main__":
    main()
