#!/usr/bin/env python3
"""Renders rank 0's share of the tiled metric frame (pt_set_tiling(BAND_ROWS, N, 0)), one frame at a
time on the whole grid, as bench.py's solo launch at N GPUs does: the process to put under
`rocprofv3 --pmc` for the per-rank counters of the N > 1 roofline (tools/gpu_share_pmc.sh).

    python tools/share_render.py --n 8 [--frames 4]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import pathtracerwithcuda_amd as pt  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--workload", default="metric")
    ap.add_argument("--group", type=int, default=1, help="frames per launch (pt_render_frames)")
    ap.add_argument("--medium-bound", action="store_true", help="pt_set_medium_bound (tolerance mode)")
    ap.add_argument("--tree", choices=list(bench.Workload.TREES), default=bench.DEFAULT_TREE)
    args = ap.parse_args()
    wl = bench.Workload(args.workload, tree=args.tree)
    r = pt.Renderer(0)
    if args.medium_bound:
        r.set_medium_bound(True)
    r.upload(wl.scene, wl.cfg)
    r.setup_frame(wl.width, wl.height)
    r.set_tiling(bench.BAND_ROWS, args.n, 0)
    bufs = None
    if args.group > 1:
        import torch

        bufs = [torch.zeros(wl.width * wl.height * 3, dtype=torch.float32, device="cuda:0")
                for _ in range(args.group)]
    for _ in range(args.frames):
        if bufs:
            r.render_frames([wl.cam] * args.group, wl.cfg, bufs, None, 1, wl.spp, write_u8=0)
        else:
            r.render(wl.cam, wl.cfg, 1, wl.spp, write_u8=0)
        r.synchronize()
    ms, n = r.kernel_time_kind(0)
    print(f"share 0 of {args.n}: {ms / max(n, 1):.3f} ms per launch of {args.group} frame(s) over {n} launches "
          f"({r.last_kernel()})")
    r.close()


if __name__ == "__main__":
    main()
