#!/usr/bin/env python3
"""PCIe-inclusive rate of the drop-in reference ABI on the bench frame: the 8 passes
of the 1920x1080 metric frame through `path_tracer_kernel` with host image buffers, one call per
pass as Core/path_tracer.cpp:40-67 makes them (each call ends with the running sum and the 8-bit
image copied back to the host, like the reference's managed memory seen from the host). The scene
is the bench scene; the first frame (scene translation and upload) is excluded.

    python tools/abi_rate.py [--frames F]
"""
import argparse
import ctypes as C
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
    args = ap.parse_args()
    wl = bench.Workload("metric")
    v, cam, cfg = wl.scene.view, wl.cam, wl.cfg
    n = wl.width * wl.height
    img = (pt._abi.Float3 * n)()
    img8 = (pt._abi.UChar3 * n)()
    scratch = [C.c_void_p() for _ in range(5)]
    lib = pt.lib()
    lib.path_tracer_kernel_memory_allocate(*[C.byref(s) for s in scratch], n)

    per_pass = [0.0] * (wl.spp + 1)

    def frame() -> None:
        for p in range(1, wl.spp + 1):
            t = time.perf_counter()
            lib.path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, n, img, img8, p,
                                   C.byref(cam), v.sky_cube_map, *scratch, v.mesh_textures, C.byref(cfg))
            per_pass[p] += time.perf_counter() - t

    frame()  # scene translation + upload on the first pass
    per_pass[:] = [0.0] * (wl.spp + 1)
    t0 = time.perf_counter()
    for _ in range(args.frames):
        frame()
    dt = (time.perf_counter() - t0) / args.frames
    lib.path_tracer_kernel_memory_free(*scratch)
    r = pt.Renderer(0)  # segments of one frame (identical for every frame: fact 2 of SURVEY.md)
    r.upload(wl.scene, wl.cfg)
    r.setup_frame(wl.width, wl.height)
    r.stats_reset()
    r.render(cam, cfg, 1, wl.spp, write_u8=0)
    r.synchronize()
    seg = r.stats()["segments"]
    r.close()
    print(json.dumps({"path": "path_tracer_kernel (reference ABI, host image buffers, one call per pass)",
                      "ms_per_frame": round(dt * 1000, 3), "mrays_per_s": round(seg / dt / 1e6, 1),
                      "ms_per_pass": [round(x / args.frames * 1000, 3) for x in per_pass[1:]],
                      "segments_per_frame": seg, "frames": args.frames}), flush=True)


if __name__ == "__main__":
    main()
