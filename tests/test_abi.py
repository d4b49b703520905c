"""CPU tests of the drop-in boundary: the library loads, exports every symbol include/*.h declares,
and the ctypes/C struct layouts equal the reference's x64 layouts."""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest

import pathtracerwithcuda_amd as pt
from pathtracerwithcuda_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//.*", "", src)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b([a-z_][a-z0-9_]*)\s*\(", src, flags=re.M):
            name = m.group(1)
            if name in ("sizeof", "offsetof", "PT_STATIC_ASSERT", "_Static_assert", "static_assert", "__attribute__"):
                continue
            names.add(name)
    return names


def test_library_exports_every_declared_symbol():
    lib = pt.lib()
    declared = declared_functions()
    assert {"path_tracer_kernel", "path_tracer_kernel_memory_allocate", "path_tracer_kernel_memory_free",
            "thread_shrink", "pt_render_passes", "pt_bvh_build"} <= declared
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, missing
    assert declared <= set(_abi.EXPORTED), sorted(declared - set(_abi.EXPORTED))


def test_struct_layouts_match_reference():
    for name, size in _abi.LAYOUT.items():
        assert C.sizeof(getattr(_abi, name)) == size, name
    assert _abi.Triangle.uv0.offset == 72 and _abi.Triangle.mat.offset == 96
    assert _abi.BvhNodeDevice.triangle_indices.offset == 40 and _abi.BvhNodeDevice.next_node_index.offset == 52
    assert _abi.RenderCamera.resolution.offset == 40
    assert _abi.Configuration.air_refraction_index.offset == 64
    assert _abi.Configuration.cuda_acceleration.offset == 92
    assert _abi.Material.medium.offset == 44 and _abi.Material.diffuse_texture_id.offset == 76


def test_configuration_defaults_follow_config_json():
    cfg = pt.configuration()
    assert (cfg.width, cfg.height, cfg.block_size, cfg.max_tracer_depth) == (1440, 900, 64, 20)
    assert abs(cfg.vector_bias_length - 0.0002) < 1e-9 and cfg.use_bilinear == 1 and cfg.use_sky == 0
    assert cfg.bvh_leaf_node_triangle_num == 1 and cfg.bvh_build == 2
    assert abs(cfg.air_refraction_index - 1.000293) < 1e-7


def test_camera_follows_view_camera_defaults():
    cam = pt.camera(640, 480)
    # eye = center + R (sin yaw cos pitch, sin pitch, cos yaw cos pitch), camera.cpp:80-98
    assert np.allclose([cam.eye.x, cam.eye.y, cam.eye.z], [0, 14 * np.sin(0.3), 14 * np.cos(0.3)], atol=1e-5)
    assert np.allclose([cam.view.x, cam.view.y, cam.view.z], [0, -np.sin(0.3), -np.cos(0.3)], atol=1e-6)
    assert cam.fov[0] == 45.0
    fy = np.degrees(np.arctan(np.tan(np.radians(45) / 2) * 480 / 640) * 2)
    assert abs(cam.fov[1] - fy) < 1e-3
    assert cam.focal_distance == 14.0 and cam.aperture_radius == 0.0


def test_no_device_fails_loudly_without_gpu():
    # On a machine without a HIP device the product must refuse, never fall back to the CPU.
    if pt.device_count() > 0:
        return
    try:
        pt.Renderer(0)
    except pt.PtError as e:
        assert "device" in str(e).lower()
    else:
        raise AssertionError("Renderer() succeeded without a device")


@pytest.mark.filterwarnings("ignore::RuntimeWarning")  # float32 overflow of the 1e30 case's helpers
@pytest.mark.parametrize("c", [0.000005, 0.0001, 0.01, 0.5, 1.0, 3.0e-20, 1.0e30, 0.0, -0.0, -1.0, float("inf"),
                               float("nan")])
def test_sqrt_le_bound_replaces_length_tests_exactly(c):
    """pt_sqrt_le_bound(c) = the largest x >= 0 with sqrtf(x) <= c: the kernels test length(v) > c as
    dot(v, v) > x (the SSS test, path_tracer_kernel.cu:460) and length(v) <= c as dot(v, v) <= x (the
    Fresnel test, fresnel.h:37, and the kill test, :612-616, written !(dot <= x) for "alive": a NaN length
    is not <= c, so a NaN throughput survives as in the reference). Both orderings are checked — each is
    false for NaN, so neither is the other's negation there — at the boundary and on random squared
    lengths (numpy's float32 sqrt is the correctly rounded sqrtf)."""
    lib = pt.lib()
    c32 = np.float32(c)
    x = np.float32(lib.pt_sqrt_le_bound(float(c32)))
    if np.isnan(c32):
        assert np.isnan(x)
        return
    rng = np.random.default_rng(7)
    d = np.concatenate([
        rng.random(20000, dtype=np.float32) * np.float32(4) * max(np.float32(abs(c32)), np.float32(1e-30)) ** 2,
        np.abs(rng.standard_normal(20000).astype(np.float32)),
        np.array([0.0, np.inf, np.nan], dtype=np.float32),
    ]).astype(np.float32)
    if x >= 0:
        near = np.array([np.nextafter(x, np.float32(-1)), x, np.nextafter(x, np.float32(np.inf))], dtype=np.float32)
        d = np.concatenate([d, near[np.isfinite(near) & (near >= 0)]]).astype(np.float32)
        assert np.sqrt(x) <= c32 and (np.isinf(x) or np.sqrt(np.nextafter(x, np.float32(np.inf))) > c32)
    with np.errstate(invalid="ignore"):
        assert np.array_equal(np.sqrt(d) > c32, d > x)
        assert np.array_equal(np.sqrt(d) <= c32, d <= x)
        # the kernel's alive test (alive_after) against the reference's kill test, NaN included
        assert np.array_equal(~(d <= x), ~(np.sqrt(d) <= c32))
        assert (~(d <= x))[np.isnan(d)].all()
