#!/usr/bin/env python3
"""Per-rank cost of the tiled frame, measured on ONE GPU: for N in 1, 2, 4, 8 the renderer is
restricted to rank r's interleaved bands (pt_set_tiling) and one frame of the metric workload is
timed for every r. The slowest rank's time against the 1-GPU frame / N is the strong-scaling
ceiling of the tiled path before any collective (the driver measures the real N-GPU runs).

    python tools/tile_scaling.py [--frames F]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import pathtracerwithcuda_amd as pt  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--counts", default="1,2,4,8")
    ap.add_argument("--inflight", type=int, default=1, help="frames in flight (one renderer context each)")
    ap.add_argument("--ranks-max", type=int, default=8, help="time at most this many ranks per N")
    ap.add_argument("--share", type=int, default=100, help="pt_set_grid_share: percent of the grid per launch")
    ap.add_argument("--order", action="store_true", help="hand out bands most expensive first (pt_set_band_order)")
    ap.add_argument("--deal", type=int, default=1, help="with --order: deal the ranked bands over this many regions (8 = PT_SHARDS)")
    ap.add_argument("--band-rows", type=int, default=0, help="rows per band (default bench.BAND_ROWS)")
    ap.add_argument("--spp", type=int, default=0,
                    help="passes per rendered frame (default the workload's 8); ms figures are per 8 passes (one "
                         "metric frame), so a 32-pass frame with PT_PASS_BATCH=32 tells what one launch for four "
                         "frames would cost")
    ap.add_argument("--group", type=int, default=1,
                    help="frames per launch (pt_render_frames): each render call renders this many frames of the "
                         "view; ms figures stay per frame")
    ap.add_argument("--total", type=int, default=0,
                    help="with --group: render this many frames in launches of at most --group frames (bench.py's "
                         "timed sequence, e.g. 20 = 8 + 8 + 4) instead of --frames full launches")
    args = ap.parse_args()
    wl = bench.Workload("metric", tree=bench.DEFAULT_TREE)
    spp = args.spp or wl.spp
    scale = wl.spp / spp  # per-frame (8-pass) figures
    rs = []
    for _ in range(args.inflight):
        r = pt.Renderer(0)
        r.set_grid_share(args.share)
        r.upload(wl.scene, wl.cfg)
        r.setup_frame(wl.width, wl.height)
        rs.append(r)
    r = rs[0]
    bufs = {}
    if args.group > 1:
        import torch

        for q in rs:
            bufs[id(q)] = [torch.zeros(wl.width * wl.height * 3, dtype=torch.float32, device="cuda:0")
                           for _ in range(args.group)]

    def draw(q, n=None) -> None:
        n = n or args.group
        if args.group > 1:
            q.render_frames([wl.cam] * n, wl.cfg, bufs[id(q)][:n], None, 1, spp, write_u8=0)
        else:
            q.render(wl.cam, wl.cfg, 1, spp, write_u8=0)

    launches = ([min(args.group, args.total - i) for i in range(0, args.total, args.group)] if args.total
                else [args.group] * args.frames)
    nframes = sum(launches)

    out = {}
    base = None
    for n in [int(x) for x in args.counts.split(",")]:
        per_rank, kern = [], []
        for k in range(min(n, args.ranks_max)):
            for q in rs:
                q.set_tiling(args.band_rows or bench.BAND_ROWS, n, k)
                if args.order:
                    q.order_bands_by_cost(wl.cam, wl.cfg, wl.spp, regions=args.deal)
                draw(q)  # warm
                q.synchronize()
                q.stats_reset()
            t0 = time.perf_counter()
            for f, g in enumerate(launches):
                draw(rs[f % len(rs)], g)
            for q in rs:
                q.synchronize()
            per_rank.append((time.perf_counter() - t0) / nframes * 1e3 * scale)
            kms, kn = r.kernel_time_kind(0)
            kern.append(kms / max(kn, 1))
        if base is None:
            base = per_rank[0]
        worst = max(per_rank)
        out[n] = {"ms_per_rank": [round(x, 3) for x in per_rank], "worst_ms": round(worst, 3),
                  "ideal_ms": round(base / n, 3),
                  "kernel_ms_worst": round(max(kern), 3), "ceiling_efficiency": round(base / n / worst, 3)}
        print(json.dumps({"n": n, **out[n]}), flush=True)
    for q in rs:
        q.close()


if __name__ == "__main__":
    main()
