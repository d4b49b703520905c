"""Host vs GPU Morton BVH build time (row f1) on the benchmark mesh sizes: 70k (config 2) and
800k (config 4) torus-knot triangles. Prints one JSON line per size; run on the GPU box.
PT_BVH_DEVICE_FINISH=0 times the device builder with its second half (bottom-up boxes, flatten) on the
host, as in round 1; the default runs it on the device (pt_bvh.hip fin_* kernels)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pathtracerwithcuda_amd as pt  # noqa: E402
from pathtracerwithcuda_amd import _abi  # noqa: E402


def tri_array(v):
    n = len(v)
    arr = (_abi.Triangle * n)()
    raw = np.zeros((n, 26), np.float32)
    raw[:, :9] = v.reshape(n, 9)
    C.memmove(arr, raw.ctypes.data, n * 104)
    return arr


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return best


for tub, rad in ((350, 100), (1000, 400)):
    v = pt.torus_knot(tub, rad).vertices.astype(np.float32)
    arr = tri_array(v)
    n = len(v)
    out = {}
    for name, dev in (("host", False), ("device", True)):
        def build():
            nodes = C.POINTER(_abi.BvhNodeDevice)()
            leaf = _abi.c_int_p()
            nn, ln = C.c_int(), C.c_int()
            if dev:
                rc = pt.lib().pt_bvh_build_device(arr, n, 0, 1, C.byref(nodes), C.byref(nn), C.byref(leaf), C.byref(ln))
            else:
                rc = pt.lib().pt_bvh_build(arr, n, 0, 1, 2, C.byref(nodes), C.byref(nn), C.byref(leaf), C.byref(ln))
            assert rc == 0
            pt.lib().pt_bvh_free(nodes, leaf)
        if dev:
            build()  # warm-up: HIP runtime, code object load
        out[name + "_ms"] = round(timed(build) * 1000, 2)
    fin = "host" if os.environ.get("PT_BVH_DEVICE_FINISH", "1") == "0" else "device"
    print(json.dumps({"triangles": n, **out, "device_second_half_on": fin}), flush=True)
