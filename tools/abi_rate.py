#!/usr/bin/env python3
"""PCIe-inclusive rate of the drop-in reference ABI on the bench frame: the 8 passes
of the 1920x1080 metric frame through `path_tracer_kernel`, one call per pass as
Core/path_tracer.cpp:40-67 makes them, on image buffers allocated as the reference allocates them
(--image managed: hipMallocManaged, Core/image.cpp:15-27) or as pageable host arrays (--image host).
Each call ends with the running sum and the 8-bit image in the caller's buffers. The scene is the
bench scene; the first frame (scene translation and upload) is excluded; the camera moves between
frames and every frame's pass 1 re-checks the scene (the reference resets pass_counter after a move).

    python tools/abi_rate.py [--frames F] [--image managed|host] [--moving]

--moving: the window while the user drags the camera (window.cpp:194-215): every call is pass 1 of a new
camera (the orbit turns by 1e-3 rad per call); reports ms per call.
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
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--image", choices=["managed", "host"], default="managed")
    ap.add_argument("--moving", action="store_true")
    args = ap.parse_args()
    wl = bench.Workload("metric")
    v, cam, cfg = wl.scene.view, wl.cam, wl.cfg
    n = wl.width * wl.height
    hip = None
    if args.image == "managed":
        hip = C.CDLL("libamdhip64.so")
        hip.hipMallocManaged.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
        hip.hipFree.argtypes = [C.c_void_p]
        pimg, pimg8 = C.c_void_p(), C.c_void_p()
        assert hip.hipMallocManaged(C.byref(pimg), n * 12, 1) == 0
        assert hip.hipMallocManaged(C.byref(pimg8), n * 3, 1) == 0
        img = C.cast(pimg, C.POINTER(pt._abi.Float3))
        img8 = C.cast(pimg8, C.POINTER(pt._abi.UChar3))
    else:
        img = (pt._abi.Float3 * n)()
        img8 = (pt._abi.UChar3 * n)()
    scratch = [C.c_void_p() for _ in range(5)]
    lib = pt.lib()
    lib.path_tracer_kernel_memory_allocate(*[C.byref(s) for s in scratch], n)

    per_pass = [0.0] * (wl.spp + 1)
    # the camera moves between frames, as it does when the reference caller resets pass_counter
    # (Core/path_tracer.cpp:101-107): every frame's pass 1 is a new render, never a repeat
    cams = [cam, pt.camera(wl.width, wl.height, yaw=1e-3, **bench.CAMERA)]

    def frame(c) -> None:
        for p in range(1, wl.spp + 1):
            t = time.perf_counter()
            lib.path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, n, img, img8, p,
                                   C.byref(c), v.sky_cube_map, *scratch, v.mesh_textures, C.byref(cfg))
            per_pass[p] += time.perf_counter() - t

    frame(cams[1])  # scene translation + upload on the first pass
    per_pass[:] = [0.0] * (wl.spp + 1)
    if args.moving:
        calls = max(8, args.frames * wl.spp)
        moving = [pt.camera(wl.width, wl.height, yaw=1e-3 * (i + 2), **bench.CAMERA) for i in range(calls)]
        t0 = time.perf_counter()
        for c in moving:
            lib.path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, n, img, img8, 1,
                                   C.byref(c), v.sky_cube_map, *scratch, v.mesh_textures, C.byref(cfg))
        dt = (time.perf_counter() - t0) / calls
        lib.path_tracer_kernel_memory_free(*scratch)
        if hip is not None:
            hip.hipFree(pimg)
            hip.hipFree(pimg8)
        print(json.dumps({"path": f"path_tracer_kernel (reference ABI, {args.image} image buffers), camera moving: "
                                  "every call is pass 1 of a new camera", "ms_per_call": round(dt * 1000, 3),
                          "calls": calls}), flush=True)
        return
    t0 = time.perf_counter()
    for f in range(args.frames):
        frame(cams[f % 2])
    dt = (time.perf_counter() - t0) / args.frames
    lib.path_tracer_kernel_memory_free(*scratch)
    if hip is not None:
        hip.hipFree(pimg)
        hip.hipFree(pimg8)
    r = pt.Renderer(0)  # segments of one frame (identical for every frame: fact 2 of SURVEY.md)
    r.upload(wl.scene, wl.cfg)
    r.setup_frame(wl.width, wl.height)
    r.stats_reset()
    r.render(cam, cfg, 1, wl.spp, write_u8=0)
    r.synchronize()
    seg = r.stats()["segments"]
    r.close()
    print(json.dumps({"path": f"path_tracer_kernel (reference ABI, {args.image} image buffers, one call per pass)",
                      "ms_per_frame": round(dt * 1000, 3), "mrays_per_s": round(seg / dt / 1e6, 1),
                      "ms_per_pass": [round(x / args.frames * 1000, 3) for x in per_pass[1:]],
                      "segments_per_frame": seg, "frames": args.frames}), flush=True)


if __name__ == "__main__":
    main()
