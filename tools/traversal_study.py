#!/usr/bin/env python3
"""STUDY TOOL: alternative BVH traversal orders replayed on the rays of the bench frame
(tools/traversal_study.c). Prints work counts and closest-hit mismatches against the reference's
preorder walk. CPU only; test infrastructure (uses the oracle)."""
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

NAMES = ["calls", "ref_nodes", "oct_nodes", "octm_nodes", "stack_boxes", "stack_pops", "oct_mismatch",
         "octm_mismatch", "anomalies", "ties", "stack_mismatch", "ref_hits", "ref_steps", "chain_steps", "chain_len",
         "skip_spec_steps", "skip_spec1_steps",
         "leaf_skip_steps", "measured_order_steps",
         "pair_merged_steps"]


def main():
    """traversal_study.py [SAMPLE [PASSES [TREE [WORKLOAD]]]]; TREE: lbvh (the reference tree) or sah<o> (PT_BVH_SAH,
    child order o, tools/tree_study.py)."""
    sample = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    tree = sys.argv[3] if len(sys.argv) > 3 else "lbvh"
    workload = sys.argv[4] if len(sys.argv) > 4 else "metric"
    so = f"/tmp/libstudy_{os.getpid()}.so"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                    "-shared", os.path.join(ROOT, "tools", "traversal_study.c"), "-o", so, "-lm"], check=True)
    oracle.build()
    oracle.VARIANTS[""] = so
    L = oracle.lib()
    L.study_stats.argtypes = [C.c_void_p]
    if tree.startswith("sah"):
        os.environ["PT_SAH_ORDER"] = tree[3:] or "0"
    wl = bench.Workload(workload, tree="sah" if tree.startswith("sah") else "lbvh")
    scene, cfg, cam = wl.scene, wl.cfg, wl.cam
    rng = np.random.default_rng(1)
    pix = np.sort(rng.choice(wl.width * wl.height, size=sample, replace=False)).astype(np.int32)
    t0 = time.time()
    oracle.render(scene.view, cam, cfg, 1, passes, pixels=pix, with_u8=False)
    st = (C.c_ulonglong * 20)()
    L.study_stats(st)
    d = dict(zip(NAMES, list(st)[:len(NAMES)]))
    reorder = os.environ.get("STUDY_REORDER")  # 1: child order from the sample's measured pass rates, 0: surface area
    if reorder is not None:
        # the re-ordered trees are walked on a second, disjoint pixel sample (the first one trained them)
        L.study_reorder(int(reorder))
        rest = np.setdiff1d(np.arange(wl.width * wl.height), pix)
        pix2 = np.sort(np.random.default_rng(2).choice(rest, size=sample, replace=False)).astype(np.int32)
        oracle.render(scene.view, cam, cfg, 1, passes, pixels=pix2, with_u8=False)
        st2 = (C.c_ulonglong * 20)()
        L.study_stats(st2)
        d2 = {k: b - a for k, a, b in zip(NAMES, list(st)[:len(NAMES)], list(st2)[:len(NAMES)])}
        c2 = max(d2["calls"], 1)
        print(f"second sample: reference-order steps per walk {d2['ref_steps'] / c2:.3f}, re-ordered "
              f"({'measured' if reorder == '1' else 'surface area'}) {d2['measured_order_steps'] / c2:.3f}")
    c = max(d["calls"], 1)
    print(f"{sample} px x {passes} passes, {time.time() - t0:.1f} s")
    for k, v in d.items():
        print(f"  {k:15s} {v:14d}  per walk {v / c:8.3f}")
    print(f"  oct/ref nodes {d['oct_nodes'] / d['ref_nodes']:.3f}  octm/ref {d['octm_nodes'] / d['ref_nodes']:.3f}"
          f"  stack pops/ref {d['stack_pops'] / d['ref_nodes']:.3f}  stack boxes/ref {d['stack_boxes'] / d['ref_nodes']:.3f}")


if __name__ == "__main__":
    main()
