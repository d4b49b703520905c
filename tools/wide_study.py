#!/usr/bin/env python3
"""STUDY TOOL: wide (collapsed) stackless BVH walks replayed on the rays of the bench frame
(tools/wide_study.c): record loads and box tests per walk against the binary two-record walk, and
closest-hit mismatches (must be 0). CPU only; test infrastructure (uses the oracle)."""
import ctypes as C
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bench  # noqa: E402
import oracle  # noqa: E402

VARIANTS = ["wide4 (2-level)", "wide4 (greedy area)", "wide8 (greedy area)"]


def main():
    sample = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
    workload = sys.argv[2] if len(sys.argv) > 2 else "metric"
    so = "/tmp/libwidestudy.so"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                    "-shared", os.path.join(ROOT, "tools", "wide_study.c"), "-o", so, "-lm"], check=True)
    oracle.build()
    oracle.VARIANTS[""] = so
    L = oracle.lib()
    L.study_stats.argtypes = [C.c_void_p]
    wl = bench.Workload(workload)
    pix = np.sort(np.random.default_rng(1).choice(wl.width * wl.height, sample, replace=False)).astype(np.int32)
    t0 = time.time()
    _, _, st0 = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 1, pixels=pix, with_u8=False)
    st = (C.c_ulonglong * 32)()
    L.study_stats(st)
    s = list(st)
    calls = s[0]
    print(f"{workload}: {sample} px, 1 pass, {st0['segments']} segments, {calls} mesh walks, {time.time() - t0:.1f} s")
    print(f"  binary: nodes/walk {s[1] / calls:.3f}  steps/walk (2 records) {s[2] / calls:.3f}  tris/walk {s[3] / calls:.3f}")
    for v, name in enumerate(VARIANTS):
        b = 4 + 4 * v
        print(f"  {name:22s} steps/walk {s[b] / calls:.3f} ({s[b] / s[2]:.3f} x binary)  with reload after a leaf "
              f"{s[b + 1] / calls:.3f} ({s[b + 1] / s[2]:.3f} x)  box tests/walk {s[b + 2] / calls:.3f} "
              f"({s[b + 2] / s[1]:.3f} x)  mismatches {s[b + 3]}")


if __name__ == "__main__":
    main()
