#!/usr/bin/env python3
"""STUDY TOOL (test infrastructure: uses the oracle). Tree quality against the reference's own BVH.

Every workload's frame is rendered by the oracle on the reference's Morton LBVH (Bvh/bvh.cpp:862-1047, the config
default MortonCodeCUDA) and on alternative trees of the same triangles, all flattened the reference's way (preorder,
skip indices, thin leaf boxes widened to the parent's) and walked by the reference's stackless walk
(path_tracer_kernel.cu:111-150):
  lbvh        the reference tree (leaf size 1, BvhLeafNodeTriangleNum)
  lbvhL<k>    the same builder with k triangles per leaf
  sah<o>      PT_BVH_SAH (binned true surface area, pt_host.cpp pt_bvh_build_sah), child order o (PT_SAH_ORDER:
              0 lower side of the split first, 1 larger surface area first, 2 more triangles first)
  sah<o>L<k>  with k triangles per leaf at most
For each: BVH nodes and triangle tests per ray segment (the oracle's own counters), and how many pixels of the float
running sum and of the 8-bit image differ from the reference tree's frame (and by how much).

    python tools/tree_study.py [--workloads metric,c2,c4,c5] [--variants lbvh,sah0,...] [--passes N] [--threads T]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bench  # noqa: E402
import oracle  # noqa: E402

PASSES = {"metric": 8, "c2": 8, "c3": 8, "c4": 8, "c5": 2}


def parse(v: str) -> tuple[str, int, int]:
    """variant -> (tree, child order, leaf size)"""
    leaf = 1
    if "L" in v:
        v, k = v.split("L")
        leaf = int(k)
    if v == "lbvh":
        return "lbvh", 0, leaf
    assert v.startswith("sah"), v
    return "sah", int(v[3:] or 0), leaf


def render(name: str, variant: str, passes: int, threads: int):
    tree, order, leaf = parse(variant)
    os.environ["PT_SAH_ORDER"] = str(order)
    t0 = time.time()
    wl = bench.Workload(name, tree=tree, leaf=leaf)
    tb = time.time() - t0
    nodes = sum(wl.scene.view.mesh_node_num[i] for i in range(wl.scene.view.mesh_num))
    t0 = time.time()
    img, img8, st = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, passes, threads=threads, with_u8=True)
    return wl, img, img8, st, {"build_s": round(tb, 2), "render_s": round(time.time() - t0, 1), "tree_nodes": nodes}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="metric,c2,c4,c5")
    ap.add_argument("--variants", default="lbvh,sah0,sah1,sah2,lbvhL2,lbvhL4,sah0L2,sah0L4")
    ap.add_argument("--passes", type=int, default=0, help="passes per frame (default: 8, C5 2)")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    oracle.build()
    rows = []
    for name in args.workloads.split(","):
        passes = args.passes or PASSES[name]
        ref = None
        for v in args.variants.split(","):
            wl, img, img8, st, info = render(name, v, passes, args.threads)
            seg = max(st["segments"], 1)
            row = {"workload": name, "variant": v, "passes": passes, "pixels": int(img.shape[0]),
                   "segments": int(st["segments"]), "nodes_per_segment": round(st["nodes"] / seg, 3),
                   "tris_per_segment": round(st["tris"] / seg, 3), **info}
            if ref is None:
                ref = (img, img8, st)
                row.update(diff_float=0, diff_u8=0, max_abs=0.0)
            else:
                same = (img.view(np.uint32) == ref[0].view(np.uint32)) | (np.isnan(img) & np.isnan(ref[0]))
                dpx = ~same.all(axis=1)
                d8 = (img8 != ref[1]).any(axis=1)
                row.update(diff_float=int(dpx.sum()), diff_u8=int(d8.sum()),
                           max_abs=float(np.nanmax(np.abs(img - ref[0]))) if dpx.any() else 0.0,
                           nodes_vs_ref=round(st["nodes"] / max(ref[2]["nodes"], 1), 4),
                           tris_vs_ref=round(st["tris"] / max(ref[2]["tris"], 1), 4),
                           segments_vs_ref=round(st["segments"] / max(ref[2]["segments"], 1), 6))
            rows.append(row)
            print(json.dumps(row), flush=True)
    if args.out:
        json.dump(rows, open(args.out, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
