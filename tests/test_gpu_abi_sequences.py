"""Randomised call sequences through the drop-in entry point, path_tracer_kernel (include/path_tracer_kernel.h),
against the oracle's pass chain, bit for bit after EVERY call.

The reference caller (Core/path_tracer.cpp:40-107, Main/window.cpp:194-215,580-588) drives one accumulation as
calls with pass_counter 1, 2, 3, ...; it restarts at 1 after every camera move and every in-place scene edit,
and F2 switches any pass to the CPU twin, which writes the same (managed) image buffers on the host. The library
behind the call keeps a translated scene, a render-ahead pass cache and host/managed/device image mirrors
(pt_runtime.cpp path_tracer_kernel, abi_render_pass), a state machine that round 4 once got wrong (a pass
served from another camera's cache). hypothesis draws sequences of:

  gpu      the next pass through path_tracer_kernel
  cpu      the next pass through the CPU twin (the oracle in the reference CPU-fallback mode: MSVC rand, libm,
           unfused arithmetic) on the same buffers — host-visible buffers only, as in the reference
  camera   the camera turns; the next pass is 1
  restart  the next pass is 1 (the caller's clear())
  material a material's diffuse colour edited in place (a sphere's or a triangle's, by pointer); next pass 1
  vertex   a triangle vertex moved in place; next pass 1

over image buffers of one kind per sequence: host (pageable), managed (hipMallocManaged, Core/image.cpp:15-27)
or device (hipMalloc). The expected state is the oracle's: the same calls applied to a numpy running sum and
8-bit image (GPU passes with the GPU kernel's arithmetic, CPU passes with the CPU twin's). The sequences are
derandomised (the same examples on every run) and sum to at least 200 path_tracer_kernel calls.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
import pathtracerwithcuda_amd as pt

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu

W, H = 40, 24
CAM = dict(pitch=0.08, radius=12.5, center=(0, 1.2, 0))
ACTIONS = ["gpu"] * 6 + ["cpu", "cpu", "camera", "restart", "material", "vertex"]


def _hip():
    h = C.CDLL("libamdhip64.so")
    h.hipMallocManaged.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    h.hipFree.argtypes = [C.c_void_p]
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    for f in (h.hipMallocManaged, h.hipMalloc, h.hipFree, h.hipMemcpy, h.hipMemset, h.hipDeviceSynchronize):
        f.restype = C.c_int
    return h


class Images:
    """The caller's image buffers of one kind, and a host view of their contents."""

    def __init__(self, hip, kind, n):
        self.hip, self.kind, self.n = hip, kind, n
        if kind == "host":
            self._f = (pt._abi.Float3 * n)()
            self._u = (pt._abi.UChar3 * n)()
            self.pf, self.pu = C.addressof(self._f), C.addressof(self._u)
        else:
            pf, pu = C.c_void_p(), C.c_void_p()
            alloc = (lambda p, b: hip.hipMallocManaged(C.byref(p), b, 1)) if kind == "managed" else \
                (lambda p, b: hip.hipMalloc(C.byref(p), b))
            assert alloc(pf, n * 12) == 0 and alloc(pu, n * 3) == 0
            self.pf, self.pu = pf.value, pu.value
            assert hip.hipMemset(self.pf, 0x7f, n * 12) == 0 and hip.hipMemset(self.pu, 7, n * 3) == 0
            assert hip.hipDeviceSynchronize() == 0

    def host_arrays(self):
        """Writable numpy views (host / managed only: the CPU twin's buffers)."""
        f = np.ctypeslib.as_array((C.c_float * (self.n * 3)).from_address(self.pf)).reshape(-1, 3)
        u = np.ctypeslib.as_array((C.c_uint8 * (self.n * 3)).from_address(self.pu)).reshape(-1, 3)
        return f, u

    def read(self):
        if self.kind != "device":
            assert self.hip.hipDeviceSynchronize() == 0
            f, u = self.host_arrays()
            return f.copy(), u.copy()
        f = np.zeros((self.n, 3), np.float32)
        u = np.zeros((self.n, 3), np.uint8)
        assert self.hip.hipMemcpy(f.ctypes.data, self.pf, self.n * 12, 2) == 0  # device to host
        assert self.hip.hipMemcpy(u.ctypes.data, self.pu, self.n * 3, 2) == 0
        return f, u

    def free(self):
        if self.kind != "host":
            self.hip.hipFree(self.pf)
            self.hip.hipFree(self.pu)


@pytest.mark.timeout(900)
def test_random_reference_abi_sequences_equal_the_oracle(require_gpu):
    hip = _hip()
    lib = pt.lib()
    n = W * H
    calls = {"gpu": 0, "cpu": 0, "seq": 0, "kinds": set()}

    @settings(max_examples=30, deadline=None, derandomize=True, database=None,
              suppress_health_check=list(HealthCheck))
    @given(kind=st.sampled_from(["host", "managed", "device"]),
           actions=st.lists(st.sampled_from(ACTIONS), min_size=14, max_size=26),
           knot=st.sampled_from([(30, 10), (40, 12)]))
    def run(kind, actions, knot):
        sc = pt.cornell_scene(pt.torus_knot(*knot), cube_length=16)
        v = sc.view
        cfg = pt.configuration(max_tracer_depth=5)
        yaw = [0.0]
        cam = pt.camera(W, H, yaw=0.0, **CAM)
        img = Images(hip, kind, n)
        scratch = [C.c_void_p() for _ in range(5)]
        lib.path_tracer_kernel_memory_allocate(*[C.byref(s) for s in scratch], n)
        want = np.zeros((n, 3), np.float32)
        want8 = np.zeros((n, 3), np.uint8)
        rng = np.random.default_rng(len(actions) * 7919 + knot[0])
        p = 1  # the next pass_counter
        calls["seq"] += 1
        calls["kinds"].add(kind)
        try:
            for step, a in enumerate(actions):
                if a == "cpu" and kind == "device":
                    a = "gpu"  # the CPU twin works on host-visible buffers only
                if a == "gpu":
                    lib.path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, n,
                                           C.cast(img.pf, C.POINTER(pt._abi.Float3)),
                                           C.cast(img.pu, C.POINTER(pt._abi.UChar3)), p, C.byref(cam),
                                           v.sky_cube_map, *scratch, v.mesh_textures, C.byref(cfg))
                    oracle.render(v, cam, cfg, p, 1, image=want, image256=want8)
                    calls["gpu"] += 1
                    p += 1
                elif a == "cpu":
                    assert hip.hipDeviceSynchronize() == 0
                    f, u = img.host_arrays()
                    oracle.render(v, cam, cfg, p, 1, rng="msvc", math="libm", arith="plain", image=f, image256=u)
                    oracle.render(v, cam, cfg, p, 1, rng="msvc", math="libm", arith="plain", image=want,
                                  image256=want8)
                    calls["cpu"] += 1
                    p += 1
                elif a == "camera":
                    yaw[0] += float(rng.uniform(-0.4, 0.4))
                    cam = pt.camera(W, H, yaw=yaw[0], **CAM)
                    p = 1
                elif a == "restart":
                    p = 1
                elif a == "material":
                    if rng.random() < 0.5 and v.sphere_num:
                        s = v.spheres[int(rng.integers(v.sphere_num))]
                        s.mat.diffuse_color.y = float(np.float32(rng.uniform(0.05, 0.95)))
                    else:
                        m = v.triangles[int(rng.integers(v.triangle_num))].mat.contents
                        m.diffuse_color.x = float(np.float32(rng.uniform(0.05, 0.95)))
                    p = 1
                elif a == "vertex":
                    t = v.triangles[int(rng.integers(v.triangle_num))]
                    t.vertex0.y = float(np.float32(t.vertex0.y + rng.uniform(-0.05, 0.05)))
                    p = 1
                if a in ("gpu", "cpu"):
                    got, got8 = img.read()
                    where = f"{kind} sequence {actions}, step {step} ({a}, pass {p - 1})"
                    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
                    assert same.all(), f"{where}: {(~same.all(axis=1)).sum()} / {n} pixels differ (float)"
                    assert np.array_equal(got8, want8), f"{where}: 8-bit image differs"
        finally:
            lib.path_tracer_kernel_memory_free(*scratch)
            img.free()

    run()
    assert calls["gpu"] >= 200, calls
    assert calls["cpu"] >= 10 and calls["kinds"] == {"host", "managed", "device"}, calls


@pytest.mark.parametrize("kind", ["host", "managed"])
@pytest.mark.parametrize("edit", [True, False])
def test_cpu_twin_pass_run_after_an_edit_is_seen_at_a_continuing_counter(require_gpu, kind, edit):
    """The F2 sequence the pass counter cannot reveal (advisor r05): GPU passes 1-2, an in-place edit (its pass-1
    reset), CPU-twin passes 1-2 on the same buffers, then the GPU again at pass 3, which continues the library's own
    last pass. The running sum the caller hands over is not the one the library returned, so the library checks the
    scene and, after an edit, redoes the call on the edited scene (its render-ahead held pass 3 of the old one).
    Without the edit the check finds the same scene and keeps the cached pass."""
    hip = _hip()
    lib = pt.lib()
    n = W * H
    sc = pt.cornell_scene(pt.torus_knot(40, 12), cube_length=16)
    v = sc.view
    cfg = pt.configuration(max_tracer_depth=5)
    cam = pt.camera(W, H, **CAM)
    img = Images(hip, kind, n)
    scratch = [C.c_void_p() for _ in range(5)]
    lib.path_tracer_kernel_memory_allocate(*[C.byref(s) for s in scratch], n)
    want = np.zeros((n, 3), np.float32)
    want8 = np.zeros((n, 3), np.uint8)

    def gpu(p):
        lib.path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, n,
                               C.cast(img.pf, C.POINTER(pt._abi.Float3)), C.cast(img.pu, C.POINTER(pt._abi.UChar3)), p,
                               C.byref(cam), v.sky_cube_map, *scratch, v.mesh_textures, C.byref(cfg))
        oracle.render(v, cam, cfg, p, 1, image=want, image256=want8)

    def cpu(p):
        assert hip.hipDeviceSynchronize() == 0
        f, u = img.host_arrays()
        for im, im8 in ((f, u), (want, want8)):
            oracle.render(v, cam, cfg, p, 1, rng="msvc", math="libm", arith="plain", image=im, image256=im8)

    try:
        gpu(1)
        gpu(2)
        if edit:  # the knot's material (every knot triangle points at it), edited in place
            m = v.triangles[v.triangle_num - 1].mat.contents
            m.diffuse_color.x = float(np.float32(0.25))
            m.diffuse_color.z = float(np.float32(0.9))
        cpu(1)
        cpu(2)
        gpu(3)
        got, got8 = img.read()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
            f"{(got != want).any(axis=1).sum()} / {n} pixels differ (float)"
        assert np.array_equal(got8, want8)
        gpu(4)  # and the library's own continuation after the redo
        got, got8 = img.read()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
        assert np.array_equal(got8, want8)
    finally:
        lib.path_tracer_kernel_memory_free(*scratch)
        img.free()
