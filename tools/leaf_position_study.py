#!/usr/bin/env python3
"""STUDY TOOL: where the passing leaves of the bench frame fall in the GPU walk's two-record steps
(tools/leaf_position_study.c). CPU only; test infrastructure (uses the oracle)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bench  # noqa: E402
import oracle  # noqa: E402

NAMES = ["walks", "steps", "leaf_first", "leaf_second", "records", "mismatch"]


def main():
    sample = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
    wl = bench.Workload(sys.argv[2] if len(sys.argv) > 2 else "metric")
    so = "/tmp/libleafpos.so"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                    "-shared", os.path.join(ROOT, "tools", "leaf_position_study.c"), "-o", so, "-lm"], check=True)
    oracle.build()
    oracle.VARIANTS[""] = so
    L = oracle.lib()
    L.study_stats.argtypes = [C.c_void_p]
    rng = np.random.default_rng(1)
    pix = np.sort(rng.choice(wl.width * wl.height, size=sample, replace=False)).astype(np.int32)
    oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 1, pixels=pix, with_u8=False)
    st = (C.c_ulonglong * 8)()
    L.study_stats(st)
    d = dict(zip(NAMES, list(st)[:len(NAMES)]))
    leaves = max(d["leaf_first"] + d["leaf_second"], 1)
    print(d)
    print(f"passing leaves first in their step: {d['leaf_first'] / leaves:.3f}; steps per walk "
          f"{d['steps'] / max(d['walks'], 1):.2f}; leaves per step {leaves / max(d['steps'], 1):.3f}")


if __name__ == "__main__":
    main()
