"""TEST INFRASTRUCTURE — Python binding of the C oracle (oracle/oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product package never does. The oracle takes the reference's own data layout (the SceneView of a
pathtracerwithcuda_amd.Scene, i.e. the pointers a reference caller passes to path_tracer_kernel).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "liboracle.so")
# "fma": the same oracle built with FMA contraction (nvcc's default), for the tolerance calibration only
VARIANTS = {"": LIB, "fma": os.path.join(HERE, "lib", "liboracle_fma.so")}

RNG = {"thrust": 0, "msvc": 1}
# "cuda" / "cuda_site": the model of the reference's hardware intrinsics (oracle_math.h), calibration only
MATH = {"cephes": 0, "libm": 1, "cuda": 2, "cuda_site": 3}
# "fma": the reference CUDA build's contraction sites as fused multiply-adds (what the HIP kernel computes);
# "plain": the same sites unfused (the MSVC-built CPU fallback; an nvcc --fmad=false build)
ARITH = {"fma": 0, "plain": 256}

_libs = {}


def build(force: bool = False, variant: str = "") -> str:
    path = VARIANTS[variant]
    srcs = [os.path.join(HERE, f) for f in ("oracle.c", "oracle_math.h", "Makefile")]
    if force or not os.path.exists(path) or any(os.path.getmtime(s) > os.path.getmtime(path) for s in srcs):
        target = os.path.relpath(path, HERE)
        subprocess.run(["make", "-s", "-C", HERE] + (["-B"] if force else []) + [target], check=True)
    return path


def lib(variant: str = "") -> C.CDLL:
    if variant not in _libs:
        build(variant=variant)
        h = C.CDLL(VARIANTS[variant])
        args = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        h.or_render.restype = C.c_int
        h.or_render.argtypes = args
        h.or_render_sig.restype = C.c_int
        h.or_render_sig.argtypes = args + [C.c_void_p]
        h.or_rng_stream.restype = None
        h.or_rng_stream.argtypes = [C.c_int, C.c_int32, C.c_int, C.c_float, C.c_float, C.c_void_p]
        h.or_hash.restype = C.c_int32
        h.or_hash.argtypes = [C.c_int32]
        h.or_gamma_u8.restype = None
        h.or_gamma_u8.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        h.or_math_eval.restype = None
        h.or_math_eval.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        _libs[variant] = h
    return _libs[variant]


def render(view, cam, cfg, first_pass: int = 1, pass_count: int = 1, pixels: np.ndarray | None = None,
           rng: str = "thrust", math: str = "cephes", threads: int = 0, with_u8: bool = True,
           image: np.ndarray | None = None, image256: np.ndarray | None = None, variant: str = "",
           signatures: bool = False, arith: str = "fma", medium_bound: bool = False):
    """Run passes first_pass..first_pass+pass_count-1 over all pixels (or the given pixel indices).

    `image` / `image256` (optional, float32 / uint8, n*3 contiguous) are the caller's running sum and
    8-bit buffers, updated in place with the reference's pass_counter semantics (a pass > 1 adds
    into the running sum): the CPU twin's view of Core/path_tracer.cpp:71-91.
    `variant` "fma" runs the build compiled with -ffp-contract=fast (calibration only); `arith` "plain"
    evaluates the contraction sites unfused (the reference CPU fallback's arithmetic). `medium_bound`:
    the product's tolerance-mode walk (PT_MEDIUM_BOUND: in-medium segments prune beyond their free flight). `signatures` adds
    stats["signatures"]: uint64 [pass_count, n], a hash of each path's decisions (hit primitive and
    branch per segment): equal signatures = same path topology.
    Returns (image float32 [n,3], image256 uint8 [n,3] or None, stats dict)."""
    L = lib(variant)
    if pixels is None:
        n = int(cam.resolution[0]) * int(cam.resolution[1])
        plist = None
    else:
        plist = np.ascontiguousarray(pixels, np.int32)
        n = len(plist)
    if image is not None:
        assert image.dtype == np.float32 and image.flags.c_contiguous and image.size == n * 3
        img = image.reshape(n, 3)
    else:
        img = np.zeros((n, 3), np.float32)
    if image256 is not None:
        assert image256.dtype == np.uint8 and image256.flags.c_contiguous and image256.size == n * 3
        img8 = image256.reshape(n, 3)
    else:
        img8 = np.zeros((n, 3), np.uint8) if with_u8 else None
    stats = (C.c_ulonglong * 6)()
    sigs = np.zeros((pass_count, n), np.uint64) if signatures else None
    rc = L.or_render_sig(view.mesh_num, C.cast(view.bvh_nodes, C.c_void_p), C.cast(view.triangles, C.c_void_p),
                     view.sphere_num, C.cast(view.spheres, C.c_void_p), C.cast(view.sky_cube_map, C.c_void_p),
                     C.cast(view.mesh_textures, C.c_void_p), C.addressof(cfg), C.addressof(cam), first_pass,
                     pass_count, plist.ctypes.data if plist is not None else None, n, img.ctypes.data,
                     img8.ctypes.data if img8 is not None else None, RNG[rng], MATH[math] | ARITH[arith] | (512 if medium_bound else 0), threads, stats,
                     sigs.ctypes.data if sigs is not None else None)
    if rc != 0:
        raise MemoryError("oracle allocation failed")
    st = {"segments": stats[0], "nodes": stats[1], "tris": stats[2], "nan_alive": stats[3],
          "nan_flight": stats[4], "inf_flight": stats[5]}
    if sigs is not None:
        st["signatures"] = sigs
    return img, img8, st


def gamma_u8(cfg, image: np.ndarray, pass_: int, math: str = "cephes") -> np.ndarray:
    """pixel_256_transform_gamma_corrected of a float running sum of `pass_` passes."""
    img = np.ascontiguousarray(image, np.float32).reshape(-1, 3)
    out = np.zeros(img.shape, np.uint8)
    lib().or_gamma_u8(C.addressof(cfg), img.ctypes.data, len(img), pass_, MATH[math], out.ctypes.data)
    return out


def rng_stream(kind: str, seed: int, n: int, a: float = 0.0, b: float = 1.0) -> np.ndarray:
    out = np.empty(n, np.float32)
    lib().or_rng_stream(RNG[kind], int(np.int32(seed)), n, a, b, out.ctypes.data)
    return out


def hash_(a: int) -> int:
    return int(lib().or_hash(int(np.int32(a))))


def hash_np(a: np.ndarray) -> np.ndarray:
    """or_hash (path_tracer_kernel.cu:35-44) over an int array: int32 wrap-around, arithmetic >>."""
    a = np.asarray(a).astype(np.int64).astype(np.uint32)
    with np.errstate(over="ignore"):
        a = (a + np.uint32(0x7ed55d16)) + (a << np.uint32(12))
        a = (a ^ np.uint32(0xc761c23c)) ^ (a.view(np.int32) >> 19).view(np.uint32)
        a = (a + np.uint32(0x165667b1)) + (a << np.uint32(5))
        a = (a + np.uint32(0xd3a2646c)) ^ (a << np.uint32(9))
        a = (a + np.uint32(0xfd7046c5)) + (a << np.uint32(3))
        a = (a ^ np.uint32(0xb55a4f09)) ^ (a.view(np.int32) >> 16).view(np.uint32)
    return a.view(np.int32)


def trace_first_draws(pass_: int, pixels: np.ndarray, depth: int) -> np.ndarray:
    """The first uniform(0, 1) draw of trace_ray_kernel's generator for (pass, pixel, depth) — the free-flight
    draw of a segment in a medium (path_tracer_kernel.cu:415,463): thrust minstd seeded with
    hash(pass) * hash(pixel) * hash(depth) (int32 wrap), one step, (x - 1) / 2^31 in float32."""
    hp = hash_np(np.asarray(pixels)).view(np.uint32).astype(np.uint64)
    k = (int(hash_np(np.array([pass_]))[0]) * int(hash_np(np.array([depth]))[0])) & 0xffffffff
    s = (hp * np.uint64(k)) & np.uint64(0xffffffff)
    x0 = s % np.uint64(2147483647)
    x0[x0 == 0] = 1
    x1 = (x0 * np.uint64(48271)) % np.uint64(2147483647)
    return (x1 - 1).astype(np.float32) / np.float32(2147483648.0)


def math_eval(which: int, mode: str, x: np.ndarray):
    x = np.ascontiguousarray(x, np.float32)
    o0 = np.empty_like(x)
    o1 = np.empty_like(x)
    lib().or_math_eval(which, MATH[mode], x.ctypes.data, len(x), o0.ctypes.data, o1.ctypes.data)
    return o0, o1


# ---- oracle/_ref: the reference's vendored third-party libraries (tinyobjloader, glm, lodepng) ----
REF_LIB = os.path.join(HERE, "_ref", "libptref.so")
REF_SRC = "/root/reference/gpu_path_tracer"
_ref = None


def build_ref(force: bool = False) -> str | None:
    """Builds oracle/_ref/libptref.so from the reference checkout's own vendored sources (Makefile
    target `ref`). Returns None when neither the checkout nor a prebuilt library is present."""
    if os.path.isdir(REF_SRC):
        subprocess.run(["make", "-s", "-C", HERE] + (["-B"] if force else []) + ["ref"], check=True)
    return REF_LIB if os.path.exists(REF_LIB) else None


def ref_lib() -> C.CDLL | None:
    global _ref
    if _ref is None:
        if build_ref() is None:
            return None
        h = C.CDLL(REF_LIB)
        fp = C.POINTER(C.POINTER(C.c_float))
        h.ptref_mesh_load.restype = C.c_int
        h.ptref_mesh_load.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p, fp, fp, fp,
                                      C.POINTER(C.POINTER(C.c_int)), C.POINTER(C.c_int)]
        h.ptref_png_decode.restype = C.c_int
        h.ptref_png_decode.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                       C.POINTER(C.POINTER(C.c_ubyte))]
        h.ptref_refit.restype = None
        h.ptref_refit.argtypes = [C.c_void_p] * 6 + [C.c_int, C.c_void_p, C.c_int] + [C.c_void_p] * 3
        h.ptref_free.restype = None
        h.ptref_free.argtypes = [C.c_void_p]
        _ref = h
    return _ref


def ref_mesh_load(path: str, position=(0, 0, 0), scale=(1, 1, 1), rotate=(0, 0, 0)):
    """Core/triangle_mesh.cpp:8-213 + :625-647 run on the real tinyobjloader and glm.
    Returns (vertices (n,3,3), normals (n,3,3), uvs (n,3,2), shape_of_triangle (n,), has_uv)."""
    h = ref_lib()
    if h is None:
        raise RuntimeError("oracle/_ref/libptref.so is not built (needs the reference checkout)")
    arr = lambda t: (C.c_float * 3)(*t)
    v, n, uv = C.POINTER(C.c_float)(), C.POINTER(C.c_float)(), C.POINTER(C.c_float)()
    sh, has_uv = C.POINTER(C.c_int)(), C.c_int()
    tri = h.ptref_mesh_load(path.encode(), arr(position), arr(scale), arr(rotate), C.byref(v), C.byref(n),
                            C.byref(uv), C.byref(sh), C.byref(has_uv))
    if tri < 0:
        raise RuntimeError(f"reference load_obj({path!r}) fails")
    try:
        V = np.ctypeslib.as_array(v, (tri * 9,)).reshape(tri, 3, 3).copy() if tri else np.zeros((0, 3, 3), np.float32)
        N = np.ctypeslib.as_array(n, (tri * 9,)).reshape(tri, 3, 3).copy() if tri else np.zeros((0, 3, 3), np.float32)
        U = np.ctypeslib.as_array(uv, (tri * 6,)).reshape(tri, 3, 2).copy() if tri else np.zeros((0, 3, 2), np.float32)
        S = np.ctypeslib.as_array(sh, (tri,)).copy() if tri else np.zeros(0, np.int32)
    finally:
        for p in (v, n, uv, sh):
            h.ptref_free(p)
    return V, N, U, S, bool(has_uv.value)


def ref_refit(init_position, init_scale, position, scale, vertices, normals, boxes):
    """glm-driven set_transform_device + update_bvh: (world vertices (n,3), normals (n,3), boxes (m,6))."""
    h = ref_lib()
    if h is None:
        raise RuntimeError("oracle/_ref/libptref.so is not built (needs the reference checkout)")
    f = lambda a: np.ascontiguousarray(a, np.float32)
    ip, isc, p, sc = f(init_position), f(init_scale), f(position), f(scale)
    v, n, b = f(vertices).reshape(-1, 3), f(normals).reshape(-1, 3), f(boxes).reshape(-1, 6)
    vo, no, bo = np.empty_like(v), np.empty_like(n), np.empty_like(b)
    h.ptref_refit(ip.ctypes.data, isc.ctypes.data, p.ctypes.data, sc.ctypes.data, v.ctypes.data, n.ctypes.data, len(v),
                  b.ctypes.data, len(b), vo.ctypes.data, no.ctypes.data, bo.ctypes.data)
    return vo, no, bo


def ref_png_decode(path: str) -> np.ndarray:
    """lodepng::decode -> (H, W, 4) uint8 RGBA."""
    h = ref_lib()
    if h is None:
        raise RuntimeError("oracle/_ref/libptref.so is not built (needs the reference checkout)")
    w, hh, px = C.c_int(), C.c_int(), C.POINTER(C.c_ubyte)()
    err = h.ptref_png_decode(path.encode(), C.byref(w), C.byref(hh), C.byref(px))
    if err:
        raise RuntimeError(f"lodepng error {err} on {path!r}")
    try:
        return np.ctypeslib.as_array(px, (hh.value, w.value, 4)).copy()
    finally:
        h.ptref_free(px)
