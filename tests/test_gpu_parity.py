"""GPU parity: the HIP path (called through the C-ABI) against the oracle on the same scene, camera,
configuration and seeds.

Tolerance: BIT-EXACT. Every random draw is keyed by (pass, pixel, depth) exactly as the reference
keys it (path_tracer_kernel.cu:324,415), both sides are compiled with contraction off, and the
transcendentals are the same documented Cephes algorithms, so the float32
running sum and the 8-bit image must match to the bit. (The distance to the CUDA build's hardware
intrinsics is calibrated separately, tests/test_oracle.py::test_libm_mode_is_close_to_cephes.)
"""
import ctypes as C

import numpy as np
import pytest

import oracle
import pathtracerwithcuda_amd as pt

pytestmark = pytest.mark.gpu

BENCH_CAM = dict(pitch=0.08, radius=12.5, center=(0, 1.2, 0))
SPHERE_CAM = dict(pitch=0.05, radius=11.0, center=(0, 1.2, 0))


def assert_bitwise(gpu, ref, what=""):
    gpu = np.asarray(gpu).reshape(ref.shape)
    if gpu.dtype == np.float32:
        same = (gpu == ref) | (np.isnan(gpu) & np.isnan(ref))
    else:
        same = gpu == ref
    bad = ~same.all(axis=-1) if same.ndim > 1 else ~same
    if bad.any():
        idx = np.flatnonzero(bad)
        d = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
        raise AssertionError(f"{what}: {bad.sum()} / {bad.size} pixels differ (first {idx[:8].tolist()}), "
                             f"max |d| {np.nanmax(d):.3g}, mean |d| {np.nanmean(d):.3g}")


@pytest.fixture(scope="module", params=["persistent", "wavefront"])
def gpu(require_gpu, request):
    """Every parity test runs under both kernel schedules (pt_set_schedule): the persistent pass kernel
    and the wavefront queues must both agree bitwise with the oracle. (Round 2's alternative kernels —
    wide walk, walker/shader regrouping, tail pool — measured slower and were removed from the library;
    they are kept as patches)"""
    r = pt.Renderer(0)
    r.set_schedule(request.param)
    assert r.schedule() == request.param
    yield r
    r.close()


def render_both(r, scene, cam, cfg, passes=1, first=1):
    r.upload(scene, cfg)
    W, H = int(cam.resolution[0]), int(cam.resolution[1])
    r.setup_frame(W, H)
    r.render(cam, cfg, first, passes, write_u8=2)
    img, img8 = r.download()
    ref, ref8, st = oracle.render(scene.view, cam, cfg, first, passes)
    return img.reshape(-1, 3), img8.reshape(-1, 3), ref, ref8, st


@pytest.mark.parametrize("which", range(9))
def test_device_math_matches_oracle_bitwise(gpu, which):
    rng = np.random.default_rng(100 + which)
    x = np.concatenate([rng.uniform(-10, 10, 50000), rng.uniform(0, 6.3, 50000), 10.0 ** rng.uniform(-38, 38, 20000),
                        [0.0, -0.0, 1.0, -1.0, 0.5, np.inf, -np.inf, np.nan, 1e-40, 88.7, -103.0]]).astype(np.float32)
    if which in (4, 5):
        x = np.clip(x, -1.2, 1.2)
    d0, d1 = gpu.math_eval_device(which, x)
    if which == 8:
        with np.errstate(all="ignore"):
            h0, h1 = np.sqrt(x), np.float32(1.0) / x
    else:
        h0, h1 = oracle.math_eval(which, "cephes", x)
        if which != 0:
            h1 = np.zeros_like(x)
    for a, b in ((d0, h0), (d1, h1)):
        same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
        assert same.all(), f"fn {which}: {(~same).sum()} mismatches, e.g. x={x[~same][:4]} gpu={a[~same][:4]} ref={b[~same][:4]}"


def test_u8_quotients_are_exact(gpu):
    """Texel bytes become pixels[i] / 255.0f (Core/texture.h:47-66); the device computes them with a
    multiply and one FMA correction instead of a division or a table: all 256 must be the quotients."""
    x = np.arange(256, dtype=np.float32)
    d0, _ = gpu.math_eval_device(9, x)
    want = x / np.float32(255.0)
    assert np.array_equal(d0.view(np.uint32), want.view(np.uint32))


def test_rcp_exact_matches_division(gpu):
    """rcp_exact (v_rcp_f32 + one Newton step) against the IEEE division 1.0f / x on the device: every
    significand in [1, 2) at several exponents and both signs, plus the guarded edges."""
    sig = (np.arange(1 << 23, dtype=np.uint32) | np.uint32(127 << 23)).view(np.float32)
    xs = [sig, -sig, sig * np.float32(2.0 ** -120), sig * np.float32(2.0 ** 100), sig * np.float32(2.0 ** -30)]
    xs.append(np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 2.0 ** -125, 2.0 ** 125, 2.0 ** -126,
                        3.4e38, 1.2e-38], np.float32))
    x = np.concatenate(xs).astype(np.float32)
    fast, div = gpu.math_eval_device(10, x)
    same = (fast.view(np.uint32) == div.view(np.uint32)) | (np.isnan(fast) & np.isnan(div))
    assert same.all(), f"{(~same).sum()} mismatches, e.g. x={x[~same][:4]} fast={fast[~same][:4]} div={div[~same][:4]}"


def test_sqrt_exact_matches_sqrtf(gpu):
    """sqrt_exact (v_sqrt_f32 + the two one-ulp residual checks, no scaling or class test on [2^-96, inf))
    against the compiler's correctly rounded sqrtf on the device: every significand at both exponent
    parities, at the guarded range's lower end and high up, plus the edges on either side of the guard."""
    sig = (np.arange(1 << 23, dtype=np.uint32) | np.uint32(127 << 23)).view(np.float32)
    xs = [sig * np.float32(2.0 ** e) for e in (0, 1, -96, -95, 100, 127)]
    xs.append(np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, -1.0, 2.0 ** -96, 2.0 ** -97,
                        np.nextafter(np.float32(2.0 ** -96), np.float32(0)), 3.4028235e38, 1.2e-38], np.float32))
    x = np.concatenate(xs).astype(np.float32)
    fast, ref = gpu.math_eval_device(11, x)
    same = (fast.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(fast) & np.isnan(ref))
    assert same.all(), f"{(~same).sum()} mismatches, e.g. x={x[~same][:4]} fast={fast[~same][:4]} ref={ref[~same][:4]}"
    with np.errstate(invalid="ignore"):
        host = np.sqrt(x)
    same = (ref.view(np.uint32) == host.view(np.uint32)) | (np.isnan(ref) & np.isnan(host))
    assert same.all(), "the device sqrtf is not the correctly rounded square root"


def test_config1_spheres_only_cornell(gpu):
    sc = pt.cornell_spheres_scene(cube_length=64)
    cfg = pt.configuration(max_tracer_depth=4)
    cam = pt.camera(64, 64, **SPHERE_CAM)
    img, img8, ref, ref8, st = render_both(gpu, sc, cam, cfg, passes=4)
    assert st["segments"] > 64 * 64 * 4
    assert_bitwise(img, ref, "float image")
    assert_bitwise(img8, ref8, "8-bit image")
    assert gpu.stats()["segments"] >= st["segments"]


def test_cornell_mesh_scene(gpu):
    sc = pt.cornell_scene(pt.torus_knot(120, 40), cube_length=128)
    cfg = pt.configuration(max_tracer_depth=8)
    cam = pt.camera(96, 54, **BENCH_CAM)
    gpu.stats_reset()
    img, img8, ref, ref8, st = render_both(gpu, sc, cam, cfg, passes=3)
    assert_bitwise(img, ref, "float image")
    assert_bitwise(img8, ref8, "8-bit image")
    assert gpu.stats()["segments"] == st["segments"]


def test_instrumented_counts_match_oracle(gpu):
    sc = pt.cornell_scene(pt.torus_knot(80, 24), cube_length=32)
    cfg = pt.configuration(max_tracer_depth=6)
    cam = pt.camera(64, 36, **BENCH_CAM)
    gpu.set_instrumented(True)
    try:
        gpu.stats_reset()
        img, _, ref, _, st = render_both(gpu, sc, cam, cfg, passes=2)
        got = gpu.stats()
    finally:
        gpu.set_instrumented(False)
    assert_bitwise(img, ref, "instrumented image")
    assert got == {"segments": st["segments"], "nodes": st["nodes"], "tris": st["tris"]}


@pytest.mark.parametrize("variant", ["ggx_dof", "sss", "glass_knot", "leaf3", "nearest_sky_noaa", "no_gamma",
                                     "textured", "air_medium", "axis_aligned_rays"])
def test_material_and_config_variants(gpu, variant):
    cfg_kw = dict(max_tracer_depth=8)
    cam_kw = dict(BENCH_CAM)
    W, H = 72, 40
    if variant == "ggx_dof":
        sc = pt.Scene()
        for i, x in enumerate(np.linspace(-2.5, 2.5, 6)):
            sc.add_sphere((x, 0.0, 0.0), 0.4, f"Micro{i + 1}")
        walls = [sc.add_material(m) for m in ("wall_white", "wall_green", "wall_red", "wall_white", "wall_white")]
        sc.add_mesh(pt.cornell_shapes(), walls, position=(0.0, -0.8, 1.0), scale=(0.1, 0.1, 0.3))
        sc.set_cube_map(pt.procedural_cube_map(64))
        sc.build()
        cam_kw.update(aperture=0.1, focal=12.5)
    elif variant == "sss":
        sc = pt.cornell_scene(pt.torus_knot(60, 16), mesh_material="DragonGreen", cube_length=32)
        cfg_kw["max_tracer_depth"] = 10
    elif variant == "glass_knot":
        sc = pt.cornell_scene(pt.torus_knot(60, 16), mesh_material="green_glass", cube_length=32)
    elif variant == "leaf3":
        sc = pt.cornell_scene(pt.torus_knot(50, 14), cube_length=32, leaf_size=3)
        cfg_kw["bvh_leaf_node_triangle_num"] = 3
    elif variant == "nearest_sky_noaa":
        sc = pt.cornell_scene(pt.torus_knot(50, 14), cube_length=0)
        cfg_kw.update(use_bilinear=0, use_sky_box=0, use_sky=1, use_anti_alias=0)
    elif variant == "no_gamma":
        sc = pt.cornell_scene(pt.torus_knot(50, 14), mesh_material="gold", cube_length=16)
        cfg_kw.update(gamma_correction=0, use_bilinear=0)
    elif variant == "textured":
        sc = pt.Scene()
        tex = (np.random.default_rng(3).uniform(0, 255, (37, 53, 4))).astype(np.uint8)
        t0 = sc.add_texture(tex)
        t1 = sc.add_texture(255 - tex[:20, :30])
        m = sc.add_material(pt.material("red", diffuse_texture_id=t0, specular_texture_id=t1))
        walls = [sc.add_material(x) for x in ("wall_white", "wall_green", "wall_red", "wall_white", "wall_white")]
        sc.add_mesh(pt.cornell_shapes(), walls, position=(0.0, -0.8, 1.0), scale=(0.1, 0.1, 0.3))
        sc.add_mesh([pt.cube_shape()], [m], position=(0.0, 1.0, 0.0), scale=(1.2, 1.2, 1.2), rotate=(20.0, 35.0, 10.0))
        sc.add_mesh([pt.cube_shape()], [sc.add_material("light")], position=(0.0, 3.1, 0.0), scale=(0.85, 0.05, 0.85))
        sc.set_cube_map(pt.procedural_cube_map(32))
        sc.build()
    elif variant == "air_medium":
        sc = pt.cornell_scene(pt.torus_knot(40, 12), cube_length=32)
        cfg_kw.update(air_absorption_coef=(0.02, 0.03, 0.05), air_reduced_scattering_coef=(0.05, 0.05, 0.05))
    elif variant == "axis_aligned_rays":
        # no jitter, yaw 0, pitch 0, odd frame: the centre column's primary rays have d.x == 0 and the
        # centre row's d.y == 0 exactly, so 1/d is infinite there (the slab test meets 0 * inf)
        sc = pt.cornell_scene(pt.torus_knot(50, 14), cube_length=32)
        cfg_kw.update(use_anti_alias=0)
        cam_kw.update(pitch=0.0)
        W, H = 73, 41
    cfg = pt.configuration(**cfg_kw)
    cam = pt.camera(W, H, **cam_kw)
    img, img8, ref, ref8, _ = render_both(gpu, sc, cam, cfg, passes=2)
    assert_bitwise(img, ref, f"{variant} float")
    assert_bitwise(img8, ref8, f"{variant} 8-bit")


def test_nan_throughput_survives_like_the_reference(gpu):
    """The kill test is length(thr) <= energy_exist_threshold (path_tracer_kernel.cu:612-616): a NaN throughput
    is NOT killed there, and the path goes on. Walls that multiply the throughput by 1e25 per diffuse bounce
    overflow it to inf within two bounces; the next wall has a zero channel, so thr * diffuse = inf * 0 = NaN
    (and a reflection off a zero-specular wall gives inf * (0 * shadow) = NaN, which the zero-specular shortcut
    must not end). The oracle counts the segments that kept a NaN path alive; the image must be bit-exact."""
    sc = pt.Scene()
    hot = sc.add_material(pt.material(((1e25, 1e25, 1e25), (0, 0, 0), (0, 0, 0), False, 0.01, 1.491, 0.0,
                                       (0, 0, 0), (0, 0, 0))))
    zero_g = sc.add_material(pt.material(((0.9, 0.0, 0.9), (0, 0, 0), (0, 0, 0), False, 0.01, 1.491, 0.0,
                                          (0, 0, 0), (0, 0, 0))))
    sc.add_mesh(pt.cornell_shapes(), [hot, zero_g, hot, zero_g, hot], position=(0.0, -0.8, 1.0), scale=(0.1, 0.1, 0.3))
    sc.add_mesh([pt.cube_shape()], [sc.add_material("light")], position=(0.0, 3.1, 0.0), scale=(0.85, 0.05, 0.85))
    sc.add_sphere((-0.9, 0.0, -0.9), 0.8, "iron")
    sc.add_sphere((1.3, 0.0, -0.4), 0.8, "glass")
    sc.set_cube_map(pt.procedural_cube_map(16))
    sc.build()
    cfg = pt.configuration(max_tracer_depth=8)
    cam = pt.camera(64, 40, **BENCH_CAM)
    img, img8, ref, ref8, st = render_both(gpu, sc, cam, cfg, passes=2)
    assert st["nan_alive"] > 1000, st
    assert_bitwise(img, ref, "NaN-throughput float")
    assert_bitwise(img8, ref8, "NaN-throughput 8-bit")


def test_leaf_skip_not_next_record(gpu):
    """A caller's node array whose leaves skip past the next record (the reference's builders never emit one,
    but path_tracer_kernel takes any array): when such a leaf's box fails, the walk jumps to its own skip index
    (path_tracer_kernel.cu:145-149), so the inline-leaf layout (which assumes the next record) must not be used.
    Every third leaf of the knot's tree skips to the end of the mesh; the image must still equal the oracle's."""
    sc = pt.cornell_scene(pt.torus_knot(40, 12), cube_length=16)
    v = sc.view
    nodes = v.bvh_nodes[2]
    count = nodes[0].next_node_index
    changed = 0
    for k in range(1, count):
        if nodes[k].is_leaf and nodes[k].next_node_index == k + 1 and k % 3 == 0:
            nodes[k].next_node_index = count
            changed += 1
    assert changed > 10
    cfg = pt.configuration(max_tracer_depth=6)
    cam = pt.camera(64, 40, **BENCH_CAM)
    img, img8, ref, ref8, _ = render_both(gpu, sc, cam, cfg, passes=2)
    if gpu.schedule() == "persistent":
        assert not gpu.last_kernel().startswith("pass_kernel_u"), gpu.last_kernel()
    assert_bitwise(img, ref, "leaf skip float")
    assert_bitwise(img8, ref8, "leaf skip 8-bit")
    std = pt.cornell_scene(pt.torus_knot(40, 12), cube_length=16)  # kept alive: the view points into it
    ref_std, _, _ = oracle.render(std.view, cam, cfg, 1, 2)
    assert not np.array_equal(ref, ref_std)  # the skips changed the walk


def _cube_at(x, y, z, s=0.18):
    c = pt.cube_shape()
    return pt.Shape((c.vertices * s + np.array([x, y, z], np.float32)).astype(np.float32), c.normals, c.uvs)


@pytest.mark.parametrize("variant", ["many_meshes", "many_materials", "many_spheres"])
def test_large_tables_and_many_meshes(gpu, variant):
    """Scenes past the pass kernel's LDS tables: more than 64 meshes (ranges beyond the LDS copy come
    from global memory), and more materials/spheres than the LDS tables hold (the launch falls back
    to pass_kernel). Bit-exact like every other scene."""
    rng = np.random.default_rng(11)
    sc = pt.Scene()
    walls = [sc.add_material(m) for m in ("wall_white", "wall_green", "wall_red", "wall_white", "wall_white")]
    sc.add_mesh(pt.cornell_shapes(), walls, position=(0.0, -0.8, 1.0), scale=(0.1, 0.1, 0.3))
    sc.add_mesh([pt.cube_shape()], [sc.add_material("light")], position=(0.0, 3.1, 0.0), scale=(0.85, 0.05, 0.85))
    if variant == "many_meshes":  # 72 meshes of one cube each, in a grid, a few materials
        mats = [sc.add_material(m) for m in ("red", "green", "gold", "diffuse_white")]
        for k in range(70):
            sc.add_mesh([_cube_at(-2.1 + 0.6 * (k % 10), -0.2 + 0.55 * (k // 10), -1.0)], [mats[k % 4]])
    elif variant == "many_materials":  # one mesh of 360 cubes, each its own material
        shapes, mats = [], []
        for k in range(360):
            shapes.append(_cube_at(-2.2 + 0.24 * (k % 20), -0.3 + 0.22 * (k // 20), -1.2, 0.08))
            d = tuple(float(v) for v in rng.uniform(0.1, 0.9, 3))
            mats.append(sc.add_material(pt.material((d, (0, 0, 0), (0.2, 0.2, 0.2), False, 0.3, 1.5, 0.0,
                                                      (0, 0, 0), (0, 0, 0)))))
        sc.add_mesh(shapes, mats)
    else:  # 320 small spheres (each with its own material record)
        for k in range(320):
            sc.add_sphere((-2.2 + 0.28 * (k % 16), -0.3 + 0.2 * (k // 16), -1.0), 0.09,
                          ("red", "gold", "glass", "iron")[k % 4])
    sc.set_cube_map(pt.procedural_cube_map(16))
    sc.build()
    cfg = pt.configuration(max_tracer_depth=5)
    cam = pt.camera(48, 32, **BENCH_CAM)
    img, img8, ref, ref8, _ = render_both(gpu, sc, cam, cfg, passes=2)
    assert_bitwise(img, ref, f"{variant} float")
    assert_bitwise(img8, ref8, f"{variant} 8-bit")


def test_full_size_pixel_subset(gpu):
    """At the benchmark size the oracle checks a random pixel subset (pixels are independent)."""
    sc = pt.cornell_scene(pt.torus_knot(), cube_length=512)
    cfg = pt.configuration(max_tracer_depth=8)
    cam = pt.camera(1920, 1080, **BENCH_CAM)
    gpu.upload(sc, cfg)
    gpu.setup_frame(1920, 1080)
    gpu.render(cam, cfg, 1, 2, write_u8=2)
    img, img8 = gpu.download()
    sel = np.random.default_rng(0).choice(1920 * 1080, 3000, replace=False).astype(np.int32)
    ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, 2, pixels=sel)
    assert_bitwise(img.reshape(-1, 3)[sel], ref, "subset float")
    assert_bitwise(img8.reshape(-1, 3)[sel], ref8, "subset 8-bit")


@pytest.fixture(scope="module")
def bench_gpu(require_gpu):
    """The schedule bench.py times (the library default: persistent pass_kernel_u, 8 passes batched)."""
    r = pt.Renderer(0)
    assert r.schedule() == "persistent"
    yield r
    r.close()


@pytest.fixture(scope="module")
def c4_workload():
    import bench
    return bench.Workload("c4")


def _render_workload(r, wl, passes=8):
    """One WHOLE frame of `passes` passes through the batched launch bench.py times, checked on every pixel
    against the oracle (float running sum and the 8-bit output of the last pass; the oracle renders the
    metric frame's 8 passes in ~2.5 s on 16 threads). Returns the launch counts by kind so the caller can
    pin the launch shape, and the oracle's stats."""
    r.upload(wl.scene, wl.cfg)
    r.setup_frame(wl.width, wl.height)
    r.stats_reset()
    r.render(wl.cam, wl.cfg, 1, passes, write_u8=2)
    r.synchronize()
    launches = {k: r.kernel_time_kind(k)[1] for k in (0, 3)}
    segments = r.stats()["segments"]
    img, img8 = r.download()
    ref, ref8, st = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, passes)
    assert_bitwise(img.reshape(-1, 3), ref, f"{wl.name} whole-frame float")
    assert_bitwise(img8.reshape(-1, 3), ref8, f"{wl.name} whole-frame 8-bit")
    assert segments == st["segments"], (segments, st["segments"])
    return launches, st


def test_c1_spheres_only_cornell_at_its_size(bench_gpu):
    """BASELINE config C1 at its own configuration (bench.py --workload c1): the spheres-only Cornell box
    (no BVH mesh), 512x512, 4 spp, 4 bounces, the 4 passes in one batched launch: all 262,144 pixels against
    the oracle, bit for bit."""
    import bench
    wl = bench.Workload("c1")
    assert (wl.width, wl.height, wl.spp, wl.depth) == (512, 512, 4, 4)
    assert wl.scene.view.mesh_num == 0 and wl.scene.view.sphere_num > 0
    launches, st = _render_workload(bench_gpu, wl, passes=4)
    assert launches == {0: 1, 3: 1}, launches
    assert st["segments"] > 512 * 512 * 4


def test_metric_frame_at_the_bench_launch_shape(bench_gpu):
    """bench.py's exact step: the metric workload (1920x1080, Cornell + 70k-triangle knot, depth 8), all
    8 passes in ONE persistent launch (batch_log2 = 3) plus one accumulate_kernel launch (its four-pass
    float4 groups, path_tracer_kernel.cu:644-651 applied pass after pass), then the 8-bit output. Every
    pixel of the frame against the oracle."""
    import bench
    wl = bench.Workload("metric")
    launches, _ = _render_workload(bench_gpu, wl, passes=8)
    assert launches == {0: 1, 3: 1}, launches


@pytest.mark.parametrize("name,passes,order", [("metric", 8, "2"), ("metric", 8, "0"), ("c2", 8, "2"), ("c4", 4, "2")])
def test_sah_tree_frames_equal_the_oracle_and_the_reference_tree(bench_gpu, monkeypatch, name, passes, order):
    """PT_BVH_SAH (pt_host.cpp pt_bvh_build_sah: the same triangles in a true-surface-area tree, flattened as the
    reference flattens its own): the HIP frame at the bench's launch shape equals the oracle walking the SAME tree on
    every pixel, bit for bit, and the stated tolerance to the reference tree's frame holds: on these
    frames the measured distance is zero, every pixel of the float running sum and of the 8-bit image equal to the
    reference LBVH's frame (tools/tree_study.py, profiles/r06/tree/), with fewer BVH nodes per segment."""
    import bench
    monkeypatch.setenv("PT_SAH_ORDER", order)
    wl = bench.Workload(name, tree="sah")
    launches, st = _render_workload(bench_gpu, wl, passes=passes)
    assert launches == {0: 1, 3: 1}, launches
    ref_wl = bench.Workload(name, tree="lbvh")
    ref, ref8, rst = oracle.render(ref_wl.scene.view, ref_wl.cam, ref_wl.cfg, 1, passes)
    img, img8 = bench_gpu.download()
    assert_bitwise(img.reshape(-1, 3), ref, f"{name} SAH frame vs the reference tree's, float")
    assert_bitwise(img8.reshape(-1, 3), ref8, f"{name} SAH frame vs the reference tree's, 8-bit")
    assert st["segments"] == rst["segments"] and st["nodes"] < rst["nodes"], (st, rst)


def test_metric_frames_grouped_as_the_bench_times_them(bench_gpu):
    """bench.py's default timed launch at N = 1: the metric frame rendered by pt_render_frames, several frames
    per launch (pass_kernel_u's MULTI instance, one accumulate per frame), each through its own camera. Every
    pixel of every frame against the oracle's frame of that camera: the bench's camera for frames 0 and 2, a
    turned camera for frame 1, so a refill that spans two frames' units must switch cameras."""
    import torch

    import bench
    wl = bench.Workload("metric")
    r = bench_gpu
    r.upload(wl.scene, wl.cfg)
    r.setup_frame(wl.width, wl.height)
    turned = pt.camera(wl.width, wl.height, yaw=0.35, **BENCH_CAM)
    cams = [wl.cam, turned, wl.cam]
    n = wl.width * wl.height * 3
    imgs = [torch.zeros(n, dtype=torch.float32, device="cuda:0") for _ in cams]
    imgs8 = [torch.zeros(n, dtype=torch.uint8, device="cuda:0") for _ in cams]
    r.stats_reset()
    r.render_frames(cams, wl.cfg, imgs, imgs8, 1, 8, write_u8=2)
    r.synchronize()
    assert r.kernel_time_kind(0)[1] == 1, "one pass launch for the three frames"
    assert "MULTI" in r.last_kernel(), r.last_kernel()
    refs = {}
    for f, cam in enumerate(cams):
        key = id(cam)
        if key not in refs:
            refs[key] = oracle.render(wl.scene.view, cam, wl.cfg, 1, 8)
        ref, ref8, _ = refs[key]
        assert_bitwise(imgs[f].cpu().numpy().reshape(-1, 3), ref, f"grouped frame {f} float")
        assert_bitwise(imgs8[f].cpu().numpy().reshape(-1, 3), ref8, f"grouped frame {f} 8-bit")


def test_twenty_frames_in_one_launch_beyond_2e28_units(bench_gpu):
    """The launch bench.py times at N >= 4 (8 N frames of a 1/N share per launch, so the driver's 20 steps are
    one launch): here the whole frame, 20 metric frames of 8 passes in ONE pass launch, 331.8 M units, past
    round 4's 2^28-unit cap, which split such a group into two launches of 4 passes. Frames 0, 9 and 19 (each
    through its own orbiting camera) equal the same camera's frame rendered alone by pt_render_passes, float
    and 8-bit, bit for bit; that single-frame path is the oracle-checked one
    (test_metric_frame_at_the_bench_launch_shape)."""
    import torch

    import bench
    wl = bench.Workload("metric")
    r = bench_gpu
    r.upload(wl.scene, wl.cfg)
    r.setup_frame(wl.width, wl.height)
    cams = [pt.camera(wl.width, wl.height, yaw=0.02 * i, **BENCH_CAM) for i in range(20)]
    n = wl.width * wl.height * 3
    assert n // 3 * 8 * len(cams) > (1 << 28)
    imgs = [torch.zeros(n, dtype=torch.float32, device="cuda:0") for _ in cams]
    imgs8 = [torch.zeros(n, dtype=torch.uint8, device="cuda:0") for _ in cams]
    r.stats_reset()
    r.render_frames(cams, wl.cfg, imgs, imgs8, 1, 8, write_u8=2)
    r.synchronize()
    assert r.kernel_time_kind(0)[1] == 1, "one pass launch for the twenty frames"
    for f in (0, 9, 19):
        r.render(cams[f], wl.cfg, 1, 8, write_u8=2)
        r.synchronize()
        solo, solo8 = r.download()
        assert_bitwise(imgs[f].cpu().numpy().reshape(-1, 3), np.asarray(solo).reshape(-1, 3), f"frame {f} float")
        assert_bitwise(imgs8[f].cpu().numpy().reshape(-1, 3), np.asarray(solo8).reshape(-1, 3), f"frame {f} 8-bit")
    del imgs, imgs8


def test_render_frames_refuses_launches_past_its_limits(bench_gpu):
    """pt_render_frames' limits fail loudly before any work: more than 2^30 units (share pixels x passes x
    frames, the kernel's 32-bit unit numbers) and more than 65535 frames (the accumulate launch's grid y)."""
    import torch

    sc = pt.cornell_scene(pt.torus_knot(20, 6), cube_length=8)
    cfg = pt.configuration(max_tracer_depth=2)
    r = bench_gpu
    r.upload(sc, cfg)
    img = torch.zeros(3, dtype=torch.float32, device="cuda:0")
    r.setup_frame(1, 1)
    cam = pt.camera(1, 1, **BENCH_CAM)
    with pytest.raises(pt.PtError, match="65535 frames"):
        r.render_frames([cam] * 65536, cfg, [img] * 65536, None, 1, 1, write_u8=0)
    big = pt.camera(4096, 4096, **BENCH_CAM)
    r.setup_frame(4096, 4096)
    imgs = [torch.zeros(3, dtype=torch.float32, device="cuda:0")] * 65  # never written: refused first
    assert 4096 * 4096 * 65 > (1 << 30)
    with pytest.raises(pt.PtError, match="too many frames"):
        r.render_frames([big] * 65, cfg, imgs, None, 1, 1, write_u8=0)
    # every frame's running sum is accumulated at the same time: frames may not share a buffer (advisor r05)
    r.setup_frame(8, 8)
    small = pt.camera(8, 8, **BENCH_CAM)
    a, b = (torch.zeros(8 * 8 * 3, dtype=torch.float32, device="cuda:0") for _ in range(2))
    a8 = torch.zeros(8 * 8 * 3, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(pt.PtError, match="share an image buffer"):
        r.render_frames([small, small], cfg, [a, a], None, 1, 1, write_u8=0)
    with pytest.raises(pt.PtError, match="share an image buffer"):
        r.render_frames([small, small], cfg, [a, b], [a8, a8], 1, 1, write_u8=2)
    r.synchronize()


def test_c2_diffuse_mesh_frame(bench_gpu):
    """BASELINE config C2 as its own workload (bench.py --workload c2): the Cornell walls and light with
    the 70k-triangle mesh, diffuse only, no spheres, 1280x720, 8 passes at the bench launch shape. Whole
    frame against the oracle."""
    import bench
    wl = bench.Workload("c2")
    assert (wl.width, wl.height, wl.spp, wl.depth) == (1280, 720, 8, 8) and wl.scene.view.sphere_num == 0
    launches, _ = _render_workload(bench_gpu, wl, passes=8)
    assert launches == {0: 1, 3: 1}, launches


def test_c3_microfacet_sky_dof_frame(bench_gpu):
    """BASELINE config C3: six GGX spheres (roughness 0.01..1, a conductor), the skybox and a thin-lens
    camera at 1920x1080, depth 8. 16 passes run as two batched launches of 8: the second batch's
    accumulate adds into the running sum the first left (path_tracer_kernel.cu:644-651, pass_counter > 1).
    Whole frame against the oracle."""
    import bench
    wl = bench.Workload("c3")
    assert wl.cam.aperture_radius > 0.0 and wl.scene.view.sphere_num == 6
    launches, _ = _render_workload(bench_gpu, wl, passes=16)
    assert launches == {0: 2, 3: 2}, launches


def test_c4_800k_sss_frame(bench_gpu, c4_workload):
    """BASELINE config C4: the 800k-triangle knot with the DragonGreen subsurface medium at 1920x1080,
    depth 8, 8 passes in one launch, whole frame against the oracle."""
    assert c4_workload.scene.triangle_count >= 800000
    launches, _ = _render_workload(bench_gpu, c4_workload, passes=8)
    assert launches == {0: 1, 3: 1}, launches


def test_medium_bound_mode_c4_frame(bench_gpu, c4_workload):
    """The medium-bounded walk (pt_set_medium_bound, a tolerance mode off by default; pt_path.h medium_bound):
    in-medium segments walk with min_t starting at their free-flight distance. The whole C4 frame through it
    equals the oracle's bounded walk bit for bit, and the bounded walk stays within the stated tolerance of
    the reference's unbounded one (measured identical on the whole frame)."""
    wl = c4_workload
    r = bench_gpu
    r.set_medium_bound(True)
    try:
        r.upload(wl.scene, wl.cfg)
        r.setup_frame(wl.width, wl.height)
        r.render(wl.cam, wl.cfg, 1, 8, write_u8=2)
        img, img8 = r.download()
        assert r.last_kernel().startswith("pass_kernel_u"), r.last_kernel()
    finally:
        r.set_medium_bound(None)
    ref, ref8, sb = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 8, medium_bound=True)
    assert_bitwise(img.reshape(-1, 3), ref, "bounded C4 float")
    assert_bitwise(img8.reshape(-1, 3), ref8, "bounded C4 8-bit")
    exact, _, se = oracle.render(wl.scene.view, wl.cam, wl.cfg, 1, 8)
    assert sb["nodes"] < 0.8 * se["nodes"], (sb["nodes"], se["nodes"])  # the walk really is bounded
    d = np.abs(ref.astype(np.float64) - exact).max(axis=1)
    assert (d <= 1e-3).mean() >= 0.998 and (d > 1e-3).mean() <= 0.001, f"{(d > 0).sum()} pixels differ"


def test_medium_bound_mode_variants(bench_gpu):
    """The bounded walk on the small subsurface scene and with a scattering air (every segment in a medium)."""
    r = bench_gpu
    for sc, cfg_kw in ((pt.cornell_scene(pt.torus_knot(60, 16), mesh_material="DragonGreen", cube_length=32),
                        dict(max_tracer_depth=10)),
                       (pt.cornell_scene(pt.torus_knot(40, 12), cube_length=32),
                        dict(max_tracer_depth=8, air_absorption_coef=(0.02, 0.03, 0.05),
                             air_reduced_scattering_coef=(0.05, 0.05, 0.05)))):
        cfg = pt.configuration(**cfg_kw)
        cam = pt.camera(72, 40, **BENCH_CAM)
        r.set_medium_bound(True)
        try:
            r.upload(sc, cfg)
            r.setup_frame(72, 40)
            r.render(cam, cfg, 1, 2, write_u8=2)
            img, img8 = r.download()
        finally:
            r.set_medium_bound(None)
        ref, ref8, st = oracle.render(sc.view, cam, cfg, 1, 2, medium_bound=True)
        assert_bitwise(img.reshape(-1, 3), ref, "bounded variant float")
        assert_bitwise(img8.reshape(-1, 3), ref8, "bounded variant 8-bit")
        # the instrumented kernel walks the bounded walk too: its node and triangle counts (the bench line's
        # counts_per_frame under --medium-bound) are the oracle's bounded counts
        r.set_medium_bound(True)
        r.set_instrumented(True)
        try:
            r.stats_reset()
            r.render(cam, cfg, 1, 2, write_u8=2)
            img_i, _ = r.download()
            got = r.stats()
        finally:
            r.set_instrumented(False)
            r.set_medium_bound(None)
        assert_bitwise(img_i.reshape(-1, 3), ref, "bounded instrumented float")
        assert got == {"segments": st["segments"], "nodes": st["nodes"], "tris": st["tris"]}


@pytest.mark.parametrize("name", ["subsurface_scattering_s", "subsurface_scattering_a", "air_sigma_s_0.5"])
def test_medium_bound_mode_reference_media(bench_gpu, tmp_path, name):
    """The medium-bounded walk beyond DragonGreen (sigma_s' = 400, mean free path 0.0025): the reference's five
    subsurface cups of subsurface_scattering_s.json (Green1 absorption-only, Green2-5 sigma_s' 5-20: mean free
    paths 0.05-0.2, longer flights that prune less and graze more) and subsurface_scattering_a.json (Absorp1-5,
    sigma_s' 5, sigma_a 0-10), and a scattering air over the metric scene (sigma_s' 0.5: every segment in a
    medium). Whole 960x540 frames, 4 passes: the HIP frame equals the oracle's bounded walk bit for bit, and the
    bounded walk stays within the stated tolerance of the reference's exact walk (measured
    identical, every pixel and every path, on the whole 1920x1080 frames: profiles/r05/medium_bound/)."""
    if name.startswith("air"):
        sc = pt.cornell_scene(pt.torus_knot(350, 100))
        cfg = pt.configuration(max_tracer_depth=8, air_absorption_coef=(0.02, 0.03, 0.05),
                               air_reduced_scattering_coef=(0.5, 0.5, 0.5))
        cam = pt.camera(960, 540, **BENCH_CAM)
    else:
        sc, cfg = _asset_scene(tmp_path, name)
        cam = pt.camera(960, 540, **ASSET_CAMS[name])
    r = bench_gpu
    r.set_medium_bound(True)
    try:
        r.upload(sc, cfg)
        r.setup_frame(960, 540)
        r.render(cam, cfg, 1, 4, write_u8=2)
        img, img8 = r.download()
        assert "FEAT=5" in r.last_kernel() or "FEAT=7" in r.last_kernel(), r.last_kernel()
    finally:
        r.set_medium_bound(None)
    ref, ref8, sb = oracle.render(sc.view, cam, cfg, 1, 4, medium_bound=True, signatures=True)
    assert_bitwise(img.reshape(-1, 3), ref, f"bounded {name} float")
    assert_bitwise(img8.reshape(-1, 3), ref8, f"bounded {name} 8-bit")
    exact, _, se = oracle.render(sc.view, cam, cfg, 1, 4, signatures=True)
    assert sb["nodes"] < 0.9 * se["nodes"], (sb["nodes"], se["nodes"])  # the walk really is bounded
    d = np.abs(ref.astype(np.float64) - exact).max(axis=1)
    flipped = (se["signatures"] != sb["signatures"]).any(axis=0)
    assert (d <= 1e-3).mean() >= 0.998 and flipped.mean() <= 0.03 and ((d > 1e-3) & ~flipped).mean() <= 0.001


def test_c5_4k_textured_depth12_frame(bench_gpu):
    """BASELINE config C5 as SURVEY.md §8(d) specifies it: the reference's vanille.obj (twice, 15 shapes each with
    vanille.json's per-shape materials and its five TGA diffuse maps) with human, cow, monkey and cup, sponza
    *_spec.tga specular maps (512^2 RGBA, 512^2 RGB, 1024^2 RGB), loaded from c5_vanille_gallery.json by the
    reference-format scene parser, at 3840x2160, depth 12, 8 passes in one launch: the whole frame (8.3 M
    pixels) against the oracle."""
    import bench
    wl = bench.Workload("c5")
    assert wl.depth == 12 and (wl.width, wl.height) == (3840, 2160)
    v = wl.scene.view
    assert v.texture_num == 8 and v.mesh_num == 8 and v.triangle_num > 100000
    assert {(v.mesh_textures[i].width, v.mesh_textures[i].height) for i in range(8)} >= {(1024, 1024), (256, 256)}
    launches, _ = _render_workload(bench_gpu, wl, passes=8)
    assert launches == {0: 1, 3: 1}, launches


def test_grid_share_changes_nothing_but_the_grid(bench_gpu):
    """pt_set_grid_share (half the grid per launch, bench.py with three frames in flight): rank 0's
    share of an 8-way tiled metric frame is the same image bit for bit."""
    import bench
    wl = bench.Workload("metric")
    r = bench_gpu
    r.upload(wl.scene, wl.cfg)
    r.setup_frame(wl.width, wl.height)
    r.set_tiling(bench.BAND_ROWS, 8, 0)
    try:
        r.render(wl.cam, wl.cfg, 1, 8, write_u8=2)
        full, full8 = r.download()
        r.render(wl.cam, wl.cfg, 1, 1, write_u8=2)  # overwrite the share with a different frame
        assert not np.array_equal(r.download()[0], full)
        r.set_grid_share(50)
        r.render(wl.cam, wl.cfg, 1, 8, write_u8=2)
        img, img8 = r.download()
    finally:
        r.set_grid_share(100)
        r.set_tiling(bench.BAND_ROWS, 1, 0)
    assert np.array_equal(img, full) and np.array_equal(img8, full8)


@pytest.mark.parametrize("share", [1, 8])
def test_band_order_changes_nothing_but_the_order(bench_gpu, share):
    """pt_set_band_order (bands handed out most expensive first, by the counters of pt_band_cost): the
    whole metric frame (share 1) and rank 0's share of an 8-way tiling are the same images bit for bit;
    the per-band counters add up to the frame's ray segments."""
    import bench
    wl = bench.Workload("metric")
    r = bench_gpu
    r.upload(wl.scene, wl.cfg)
    r.setup_frame(wl.width, wl.height)
    r.set_tiling(bench.BAND_ROWS, share, 0)
    try:
        r.stats_reset()
        r.render(wl.cam, wl.cfg, 1, 8, write_u8=2)
        r.synchronize()
        segments = r.stats()["segments"]
        full, full8 = r.download()
        order = r.order_bands_by_cost(wl.cam, wl.cfg, 8)
        n, partial = r.band_count()
        assert sorted(order) == list(range(n)) and order != list(range(n))
        r.measure_band_cost(True)
        r.render(wl.cam, wl.cfg, 1, 1, write_u8=2)  # overwrite with a different frame, counting
        assert not np.array_equal(r.download()[0], full)
        one_pass = sum(r.band_cost())
        r.measure_band_cost(False)
        r.stats_reset()
        r.render(wl.cam, wl.cfg, 1, 8, write_u8=2)
        r.synchronize()
        assert r.stats()["segments"] == segments
        img, img8 = r.download()
        assert 0 < one_pass < segments
    finally:
        r.set_band_order(None)
        r.set_tiling(bench.BAND_ROWS, 1, 0)
    assert np.array_equal(img, full) and np.array_equal(img8, full8)
    with pytest.raises(RuntimeError):
        bad = list(order)
        bad[0] = bad[1]
        r.set_tiling(bench.BAND_ROWS, share, 0)
        r.set_band_order(bad)
    r.set_tiling(bench.BAND_ROWS, 1, 0)


@pytest.mark.parametrize("bands", [4, 8])
def test_c4_band_tiling_partitions_the_frame(bench_gpu, c4_workload, bands):
    """The multi-GPU partition on the C4 scene at the bench's 8-row bands: every rank's share rendered
    with pt_set_tiling equals the single-context frame on its rows, bit for bit, and the shares cover
    the frame."""
    wl = c4_workload
    r = bench_gpu
    r.upload(wl.scene, wl.cfg)
    r.setup_frame(wl.width, wl.height)
    r.render(wl.cam, wl.cfg, 1, 8, write_u8=0)
    full, _ = r.download()
    owned = np.zeros(wl.height, bool)
    try:
        for k in range(bands):
            r.set_tiling(8, bands, k)
            r.render(wl.cam, wl.cfg, 1, 8, write_u8=0)
            part, _ = r.download()
            rows = pt.owned_rows(wl.height, 8, bands, k)
            assert not owned[rows].any()
            owned[rows] = True
            assert np.array_equal(part[rows], full[rows]), f"band owner {k} of {bands}"
    finally:
        r.set_tiling(1, 1, 0)
    assert owned.all()


def test_schedule_switch_on_one_context(require_gpu):
    """persistent -> wavefront (a larger frame grows the wavefront buffers) -> persistent on ONE context:
    each render equals the oracle (the batched pass buffer must survive the wavefront schedule's growth)."""
    sc = pt.cornell_scene(pt.torus_knot(40, 12), cube_length=16)
    cfg = pt.configuration(max_tracer_depth=5)
    r = pt.Renderer(0)
    try:
        for sched, (w, h) in (("persistent", (48, 32)), ("wavefront", (96, 64)), ("persistent", (48, 32)),
                              ("persistent", (96, 64))):
            r.set_schedule(sched)
            cam = pt.camera(w, h, **BENCH_CAM)
            img, img8, ref, ref8, _ = render_both(r, sc, cam, cfg, passes=4)
            assert_bitwise(img, ref, f"{sched} {w}x{h} float")
            assert_bitwise(img8, ref8, f"{sched} {w}x{h} 8-bit")
    finally:
        r.close()


def test_band_tiling_partitions_the_frame(gpu):
    sc = pt.cornell_scene(pt.torus_knot(60, 16), cube_length=32)
    cfg = pt.configuration(max_tracer_depth=6)
    cam = pt.camera(64, 45, **BENCH_CAM)
    gpu.upload(sc, cfg)
    gpu.setup_frame(64, 45)
    gpu.render(cam, cfg, 1, 2)
    full, _ = gpu.download()
    acc = np.zeros_like(full)
    owned = np.zeros(full.shape[:2], bool)
    for k in range(3):
        gpu.setup_frame(64, 45)
        gpu.render(cam, cfg, 1, 1)   # overwrite everything first (pass 1 semantics on all rows)
        gpu.set_tiling(8, 3, k)
        gpu.render(cam, cfg, 1, 2)   # owned rows now hold the 2-pass sum
        part, _ = gpu.download()
        rows = [y for y in range(45) if (y // 8) % 3 == k]
        acc[rows] = part[rows]
        owned[rows] = True
        gpu.set_tiling(1, 1, 0)
    assert owned.all()
    assert np.array_equal(acc, full)


@pytest.mark.parametrize("case", ["sky_only", "spheres_only_sky_off", "depth0", "depth1", "tiny_2x2", "odd_pass_range"])
def test_edge_cases(gpu, case):
    """Degenerate inputs of the pass: a scene with nothing but the sky, no background at all, zero and
    one bounce, a 2x2 frame, and a continuation range of passes that is not a power of two (3..9: the
    launch splits it into batches of 4, 2 and 1 passes)."""
    sc = pt.cornell_scene(pt.torus_knot(30, 10), cube_length=16)
    cfg_kw = dict(max_tracer_depth=6)
    W, H, first, passes = 24, 18, 1, 2
    if case == "sky_only":
        s0 = pt.Scene()
        s0.set_cube_map(pt.procedural_cube_map(16))
        sc = s0.build()
    elif case == "spheres_only_sky_off":
        sc = pt.cornell_spheres_scene(cube_length=0)
        cfg_kw.update(use_sky_box=0, use_sky=0)
    elif case == "depth0":
        cfg_kw["max_tracer_depth"] = 0
    elif case == "depth1":
        cfg_kw["max_tracer_depth"] = 1
    elif case == "tiny_2x2":
        W, H = 2, 2
    elif case == "odd_pass_range":
        first, passes = 3, 7
    cfg = pt.configuration(**cfg_kw)
    cam = pt.camera(W, H, **BENCH_CAM)
    gpu.upload(sc, cfg)
    gpu.setup_frame(W, H)
    if first > 1:
        gpu.render(cam, cfg, 1, first - 1, write_u8=0)
    gpu.render(cam, cfg, first, passes, write_u8=2)
    img, img8 = gpu.download()
    ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, first - 1 + passes)
    assert_bitwise(img.reshape(-1, 3), ref, f"{case} float")
    assert_bitwise(img8.reshape(-1, 3), ref8, f"{case} 8-bit")


@pytest.mark.parametrize("case", ["one_launch", "odd_range", "tiled", "grid_share", "depth0", "tiny_frames"])
def test_render_frames_equal_separate_frames(gpu, case):
    """pt_render_frames: several frames, each through its own camera, in one pass launch per batch of passes
    (the persistent schedule; the wavefront schedule renders them one after another). Every frame is the
    oracle's frame of its camera bit for bit, 8-bit output included, and frame f's radiances are summed into
    its own image. Cases: one 8-pass launch; a continuation range 2..4 (batches of 2 and 1, the one-pass launch
    through pass_rad too); a 3-band share (rows of band 1 only); a 45 % grid; max_depth 0 (every path ends at
    generation, through the MULTI instance's finish); 4x2 frames (8 pixels x 8 passes = 64 units: one chunk can
    hold units of several frames).

    The frames' units follow each other (frame f's unit u is f * units_per_frame + u). A wave's chunk of 64 units
    (pt_work.h) is generated whole into the wave's LDS ring (pass_kernel_u gen_ring_fill); the camera is read
    through the scalar cache, so a chunk that holds units of two or more frames is generated frame by frame (the
    lanes of the first pending lane's frame, then the next). With W x H = 70 x 45 and 8 passes a frame is 25,200
    units, not a multiple of 64, so some chunk straddles every frame boundary (asserted below)."""
    import torch

    sc = pt.cornell_scene(pt.torus_knot(60, 16), cube_length=32)
    cfg = pt.configuration(max_tracer_depth=0 if case == "depth0" else 6)
    W, H = (4, 2) if case == "tiny_frames" else (70, 45)
    cams = [pt.camera(W, H, yaw=y, **BENCH_CAM) for y in (0.0, 0.4, -0.7)]
    first, count = (2, 3) if case == "odd_range" else (1, 8)
    if case in ("one_launch", "depth0"):
        assert (W * H * count) % 64 != 0  # a chunk spans the boundary between frames 0 and 1
    gpu.upload(sc, cfg)
    gpu.setup_frame(W, H)
    if case == "tiled":
        gpu.set_tiling(8, 3, 1)
    if case == "grid_share":
        gpu.set_grid_share(45)
    try:
        imgs = [torch.full((H * W * 3,), 7.0, dtype=torch.float32, device="cuda:0") for _ in cams]
        imgs8 = [torch.zeros((H * W * 3,), dtype=torch.uint8, device="cuda:0") for _ in cams]
        if first > 1:
            gpu.render_frames(cams, cfg, imgs, imgs8, 1, first - 1, write_u8=0)
        gpu.render_frames(cams, cfg, imgs, imgs8, first, count, write_u8=2)
        gpu.synchronize()
        rows = [y for y in range(H) if (y // 8) % 3 == 1] if case == "tiled" else list(range(H))
        for f, cam in enumerate(cams):
            ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, first - 1 + count)
            img = imgs[f].cpu().numpy().reshape(H, W, 3)[rows]
            img8 = imgs8[f].cpu().numpy().reshape(H, W, 3)[rows]
            assert_bitwise(img.reshape(-1, 3), ref.reshape(H, W, 3)[rows].reshape(-1, 3), f"{case} frame {f} float")
            assert_bitwise(img8.reshape(-1, 3), ref8.reshape(H, W, 3)[rows].reshape(-1, 3), f"{case} frame {f} 8-bit")
            if case == "tiled":  # rows outside the share untouched
                other = [y for y in range(H) if y not in rows]
                assert (imgs[f].cpu().numpy().reshape(H, W, 3)[other] == 7.0).all()
    finally:
        gpu.set_tiling(1, 1, 0)
        gpu.set_grid_share(100)


@pytest.mark.parametrize("inflight", [2, 3, 5])
def test_frames_in_flight_equal_one_at_a_time(require_gpu, inflight):
    """bench.py's frame pipeline: frames queued on several contexts with no host sync between them
    (TiledFrame.launch) each end with the image of a frame rendered on its own, bit for bit; with F >= 3
    contexts each launches on 1 / (F - 1) of the grid and the last frame on the whole grid, as bench.py
    does (three for the whole frame, five for a tiled share)."""
    sc = pt.cornell_scene(pt.torus_knot(80, 24), cube_length=32)
    cfg = pt.configuration(max_tracer_depth=8)
    cam = pt.camera(96, 64, **BENCH_CAM)
    ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, 4)
    rs = [pt.Renderer(0) for _ in range(inflight)]
    try:
        frames = []
        for q in rs:
            q.upload(sc, cfg)
            if inflight >= 3:
                q.set_grid_share(100 // (inflight - 1))
            frames.append(pt.TiledFrame(q, 96, 64))
        n = 2 * inflight + 1
        for i in range(n):
            if inflight >= 3 and i == n - 1:
                rs[i % inflight].set_grid_share(100)
            frames[i % inflight].launch(cam, cfg, 4)
        for f in frames:
            f.synchronize()
        for q in rs:
            img, img8 = q.download()
            assert_bitwise(img.reshape(-1, 3), ref, "in-flight frame")
            assert np.array_equal(img8.reshape(-1, 3), ref8)
    finally:
        for q in rs:
            q.close()


def test_reference_abi_path_tracer_kernel(gpu):
    """The drop-in entry point with host buffers, pass by pass, as Core/path_tracer.cpp:40-67 calls it."""
    sc = pt.cornell_scene(pt.torus_knot(50, 14), cube_length=32)
    cfg = pt.configuration(max_tracer_depth=5)
    cam = pt.camera(40, 30, **BENCH_CAM)
    n = 40 * 30
    img = (pt._abi.Float3 * n)()
    img8 = (pt._abi.UChar3 * n)()
    scratch = [C.c_void_p() for _ in range(5)]
    lib = pt.lib()
    lib.path_tracer_kernel_memory_allocate(*[C.byref(s) for s in scratch], n)
    v = sc.view
    for p in (1, 2, 3):
        lib.path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, n, img, img8, p,
                               C.byref(cam), v.sky_cube_map, *scratch, v.mesh_textures, C.byref(cfg))
    lib.path_tracer_kernel_memory_free(*scratch)
    got = np.frombuffer(img, np.float32).reshape(-1, 3)
    got8 = np.frombuffer(img8, np.uint8).reshape(-1, 3)
    ref, ref8, _ = oracle.render(v, cam, cfg, 1, 3)
    assert_bitwise(got, ref, "ABI float")
    assert_bitwise(got8, ref8, "ABI 8-bit")


def _hip_runtime():
    h = C.CDLL("libamdhip64.so")
    h.hipMallocManaged.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    h.hipMallocManaged.restype = C.c_int
    h.hipFree.argtypes = [C.c_void_p]
    h.hipFree.restype = C.c_int
    h.hipDeviceSynchronize.restype = C.c_int
    return h


def test_reference_abi_alternates_with_cpu_twin_on_managed_buffers(require_gpu):
    """Core/path_tracer.cpp:40-91 picks the GPU entry or the CPU twin path_tracer_cpu per pass, on the
    SAME managed image (Core/image.cpp:15-27) and scratch (path_tracer_kernel.cu:782-796) buffers. Here
    passes 1, 3, 4 run through path_tracer_kernel and passes 2, 5 are the CPU twin (the oracle in the
    reference CPU-fallback mode: MSVC rand, libm, unfused arithmetic) writing the managed buffers on the host. Every GPU
    pass must add into what the host left there: the result equals the same five-pass chain run by
    the oracle alone, bit for bit."""
    sc = pt.cornell_scene(pt.torus_knot(50, 14), cube_length=32)
    cfg = pt.configuration(max_tracer_depth=5)
    cam = pt.camera(40, 30, **BENCH_CAM)
    n = 40 * 30
    hip = _hip_runtime()
    lib = pt.lib()
    pimg, pimg8 = C.c_void_p(), C.c_void_p()
    assert hip.hipMallocManaged(C.byref(pimg), n * 12, 1) == 0
    assert hip.hipMallocManaged(C.byref(pimg8), n * 3, 1) == 0
    scratch = [C.c_void_p() for _ in range(5)]
    lib.path_tracer_kernel_memory_allocate(*[C.byref(s) for s in scratch], n)
    try:
        img = np.ctypeslib.as_array((C.c_float * (n * 3)).from_address(pimg.value))
        img8 = np.ctypeslib.as_array((C.c_uint8 * (n * 3)).from_address(pimg8.value))
        img[:] = np.nan  # pass 1 must overwrite whatever the buffers held
        img8[:] = 7
        # the scratch is host-accessible, as the CPU twin uses it (path_tracer_cpu.cpp:244-262)
        for s, nb in zip(scratch, (12, 12, 24, 4, 24)):
            a = np.ctypeslib.as_array((C.c_uint8 * (n * nb)).from_address(s.value))
            a[:] = 0xA5
            assert a[-1] == 0xA5
        v = sc.view
        want = np.zeros((n, 3), np.float32)
        want8 = np.zeros((n, 3), np.uint8)
        for p, backend in ((1, "gpu"), (2, "cpu"), (3, "gpu"), (4, "gpu"), (5, "cpu")):
            if backend == "gpu":
                lib.path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, n,
                                       C.cast(pimg, C.POINTER(pt._abi.Float3)), C.cast(pimg8, C.POINTER(pt._abi.UChar3)),
                                       p, C.byref(cam), v.sky_cube_map, *scratch, v.mesh_textures, C.byref(cfg))
                oracle.render(v, cam, cfg, p, 1, image=want, image256=want8)
            else:
                assert hip.hipDeviceSynchronize() == 0
                oracle.render(v, cam, cfg, p, 1, rng="msvc", math="libm", arith="plain", image=img, image256=img8)
                oracle.render(v, cam, cfg, p, 1, rng="msvc", math="libm", arith="plain", image=want, image256=want8)
        assert hip.hipDeviceSynchronize() == 0
        assert_bitwise(img.reshape(-1, 3), want, "alternating GPU/CPU float")
        assert_bitwise(img8.reshape(-1, 3), want8, "alternating GPU/CPU 8-bit")
        # and the chain differs from an all-GPU one (the CPU passes really were picked up)
        gpu_only, _, _ = oracle.render(v, cam, cfg, 1, 5)
        assert not np.array_equal(gpu_only, want)
    finally:
        lib.path_tracer_kernel_memory_free(*scratch)
        hip.hipFree(pimg)
        hip.hipFree(pimg8)


def test_reference_abi_pass_cache_follows_camera_and_passes(require_gpu):
    """The reference ABI renders passes ahead in batched launches and serves later calls from them
    (pt_runtime.cpp abi_render_pass): every call must still equal the oracle's pass chain, when the camera
    moves (the cache is keyed by the camera bytes), when the pass counter restarts, and past the end of a
    batch (passes 1..10 cross the two 4-pass slots into a new batch)."""
    sc = pt.cornell_scene(pt.torus_knot(40, 12), cube_length=16)
    cfg = pt.configuration(max_tracer_depth=5)
    cams = [pt.camera(48, 32, **BENCH_CAM), pt.camera(48, 32, yaw=0.3, **BENCH_CAM)]
    n = 48 * 32
    img = (pt._abi.Float3 * n)()
    img8 = (pt._abi.UChar3 * n)()
    scratch = [C.c_void_p() for _ in range(5)]
    lib = pt.lib()
    lib.path_tracer_kernel_memory_allocate(*[C.byref(s) for s in scratch], n)
    v = sc.view
    try:
        for cam_i, passes in ((0, 3), (1, 2), (0, 10), (0, 1), (1, 6)):
            cam = cams[cam_i]
            want = np.zeros((n, 3), np.float32)
            want8 = np.zeros((n, 3), np.uint8)
            for p in range(1, passes + 1):
                lib.path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, n, img, img8, p,
                                       C.byref(cam), v.sky_cube_map, *scratch, v.mesh_textures, C.byref(cfg))
                oracle.render(v, cam, cfg, p, 1, image=want, image256=want8)
                assert_bitwise(np.frombuffer(img, np.float32).reshape(-1, 3), want, f"camera {cam_i} pass {p} float")
                assert_bitwise(np.frombuffer(img8, np.uint8).reshape(-1, 3), want8, f"camera {cam_i} pass {p} 8-bit")
    finally:
        lib.path_tracer_kernel_memory_free(*scratch)


def test_reference_abi_sees_in_place_edits(require_gpu):
    """The reference ABI keeps the resident scene when a pass-1 call re-sends identical content, and must
    re-read it after an in-place edit (the reference's editor writes materials and spheres into the same
    managed buffers, then resets pass_counter): the edited frame equals the oracle's, and so does the
    unedited one rendered again after it."""
    sc = pt.cornell_scene(pt.torus_knot(40, 12), cube_length=16)
    cfg = pt.configuration(max_tracer_depth=5)
    cam = pt.camera(32, 24, **BENCH_CAM)
    n = 32 * 24
    img = (pt._abi.Float3 * n)()
    img8 = (pt._abi.UChar3 * n)()
    scratch = [C.c_void_p() for _ in range(5)]
    lib = pt.lib()
    lib.path_tracer_kernel_memory_allocate(*[C.byref(s) for s in scratch], n)
    v = sc.view

    def frame(passes=2):
        for p in range(1, passes + 1):
            lib.path_tracer_kernel(v.mesh_num, v.bvh_nodes, v.triangles, v.sphere_num, v.spheres, n, img, img8, p,
                                   C.byref(cam), v.sky_cube_map, *scratch, v.mesh_textures, C.byref(cfg))
        return np.frombuffer(img, np.float32).reshape(-1, 3).copy()

    try:
        base = frame()
        assert_bitwise(frame(), base, "unchanged scene, second frame")
        old = v.spheres[0].mat.diffuse_color.x, v.spheres[0].radius
        v.spheres[0].mat.diffuse_color.x = 0.123
        v.spheres[0].radius = old[1] * 1.3
        edited = frame()
        ref, _, _ = oracle.render(v, cam, cfg, 1, 2)
        assert_bitwise(edited, ref, "after in-place edit")
        assert not np.array_equal(edited, base)
        v.spheres[0].mat.diffuse_color.x, v.spheres[0].radius = old
        assert_bitwise(frame(), base, "edit undone")
    finally:
        lib.path_tracer_kernel_memory_free(*scratch)


def test_thread_shrink_matches_stable_remove_if(gpu):
    import torch
    rng = np.random.default_rng(5)
    for n in (1, 63, 64, 1000, 300001):
        a = rng.integers(0, 10**6, n).astype(np.int32)
        a[rng.random(n) < 0.4] = -1
        t = torch.tensor(a, device="cuda")
        torch.cuda.synchronize()
        k = pt.lib().thread_shrink(C.c_void_p(t.data_ptr()), n)
        want = a[a >= 0]
        assert k == len(want)
        assert np.array_equal(t[:k].cpu().numpy(), want)


@pytest.mark.parametrize("name,bvh", [("cornell_box_simple", 2), ("depth_of_view", 2), ("fresnel", 2),
                                      ("micro_surface", 2), ("refractive_index", 2), ("tex_cube", 2),
                                      ("cornell_box_simple", 0), ("fresnel", 0)])
def test_reference_scene_files(gpu, tmp_path, name, bvh):
    """The reference's own scene JSONs (tests/golden/res), loaded by the C++ scene parser with the
    config.json of the checkout, built with the configured builder (MortonCodeCUDA on the GPU or
    NaiveCPU), rendered at the default orbit camera: bit-exact against the oracle."""
    from test_loader import make_root

    root = make_root(tmp_path)
    cfg = pt.load_config(str(root / "res" / "configuration" / "config.json"))
    cfg.bvh_build = bvh
    cfg.max_tracer_depth = 6
    sc = pt.load_scene(str(root / "res" / "scene" / f"{name}.json"), root_dir=str(root), config=cfg)
    kw = dict(BENCH_CAM) if name.startswith("cornell") else {}
    if name == "depth_of_view":
        kw.update(aperture=0.15, focal=13.0)
    cam = pt.camera(64, 40, **kw)
    img, img8, ref, ref8, _ = render_both(gpu, sc, cam, cfg, passes=2)
    assert_bitwise(img, ref, f"{name} float")
    assert_bitwise(img8, ref8, f"{name} 8-bit")


ASSET_CAMS = {"vanille": dict(center=(0, 0, 0), radius=70.0, pitch=0.1),
              "vanille_nude": dict(center=(0, 0, 0), radius=70.0, pitch=0.1),
              "subsurface_scattering_s": dict(center=(0, 0.8, 0), radius=11.0, pitch=0.1),
              "subsurface_scattering_a": dict(center=(0, 0.8, 0), radius=11.0, pitch=0.1),
              "dinosaur": dict(center=(0, 0, 0), radius=16.0, pitch=0.15, yaw=1.2)}


def _asset_scene(tmp_path, name, depth=8):
    from test_loader import make_root

    root = make_root(tmp_path, assets=True)
    cfg = pt.load_config(str(root / "res" / "configuration" / "config.json"))
    cfg.max_tracer_depth = depth
    sc = pt.load_scene(str(root / "res" / "scene" / f"{name}.json"), root_dir=str(root), config=cfg,
                       background="res\\texture\\lobby", background_format="bmp")
    return sc, cfg


@pytest.mark.parametrize("name", list(ASSET_CAMS))
def test_reference_asset_scene_frames(gpu, tmp_path, name):
    """The reference's own scenes over its own assets (tests/golden/ref_assets.tar.xz): vanille.json (25,786
    triangles in 15 shapes with per-shape materials, vanille.json:102, and five TGA diffuse maps of 256^2-1024^2),
    vanille_nude.json (its missing c595_00.tga generated), subsurface_scattering_s.json (five 24k-triangle cups:
    Green1 is absorption-only, sigma_s' = 0, so its free flights are -log(u) / 0 = +inf; Green2-5 scatter with
    sigma_s' 5-20), subsurface_scattering_a.json and dinosaur.json; the lobby BMP skybox where theirs is missing
    (yokohama) or JPEG (lycksele). Whole 320x180 frames, 2 passes, depth 8, under both schedules: bit-exact."""
    sc, cfg = _asset_scene(tmp_path, name)
    cam = pt.camera(320, 180, **ASSET_CAMS[name])
    img, img8, ref, ref8, st = render_both(gpu, sc, cam, cfg, passes=2)
    assert_bitwise(img, ref, f"{name} float")
    assert_bitwise(img8, ref8, f"{name} 8-bit")
    if name == "subsurface_scattering_s":
        assert st["inf_flight"] > 1000, st  # segments inside Green1 reached the sigma_s' = 0 branch


def test_absorption_only_medium_nan_free_flight(gpu, tmp_path):
    """The free flight of path_tracer_kernel.cu:463-466 over sigma_s' = 0 when the draw is exactly 1.0f:
    -__logf(1.0f) / 0 = -0 / 0 = NaN, which is never below min_t, so the segment is attenuated over min_t and
    shades its hit (the +inf case of any other draw goes the same way). subsurface_scattering_s.json with an
    absorption-only air (sigma_a > 0, sigma_s' = 0, Green1's kind of medium) makes every segment draw a free
    flight; the pass is chosen so that one pixel's depth-0 draw rounds to 1.0f (the oracle's restatement of the
    generator finds it: probability ~3e-8 per draw). Passes 1 and that pass, bit-exact, with the oracle counting
    the NaN flight."""
    sc, cfg = _asset_scene(tmp_path, "subsurface_scattering_s", depth=6)
    cfg.air_absorption_coef = pt._abi.Float3(0.02, 0.03, 0.013)
    cfg.air_reduced_scattering_coef = pt._abi.Float3(0.0, 0.0, 0.0)
    W, H = 320, 180
    cam = pt.camera(W, H, **ASSET_CAMS["subsurface_scattering_s"])
    pixels = np.arange(W * H)
    p = next(p for p in range(2, 100000) if (oracle.trace_first_draws(p, pixels, 0) == 1.0).any())
    hit = np.flatnonzero(oracle.trace_first_draws(p, pixels, 0) == 1.0)
    gpu.upload(sc, cfg)
    gpu.setup_frame(W, H)
    gpu.render(cam, cfg, 1, 1, write_u8=0)
    gpu.render(cam, cfg, p, 1, write_u8=2)
    img, img8 = gpu.download()
    ref = np.zeros((W * H, 3), np.float32)
    ref8 = np.zeros((W * H, 3), np.uint8)
    oracle.render(sc.view, cam, cfg, 1, 1, image=ref, image256=ref8)
    _, _, st = oracle.render(sc.view, cam, cfg, p, 1, image=ref, image256=ref8)
    assert st["nan_flight"] >= len(hit) >= 1, (p, hit, st)
    assert st["inf_flight"] > 0, st
    assert_bitwise(img.reshape(-1, 3), ref, f"pass {p} float")
    assert_bitwise(img8.reshape(-1, 3), ref8, f"pass {p} 8-bit")


def test_device_refit_equals_the_edited_scene(require_gpu):
    """Interactive edits (f4). pt_mesh_set_transform re-transforms an attached mesh's resident triangles
    and refits its resident boxes on the device (Core/triangle_mesh.cpp:271-328, Bvh/bvh.cpp:332-356);
    the host builder's set_transform makes the same edit to the reference-layout scene. After each of
    several moves of two meshes the device-refitted context renders exactly the oracle's image of the
    edited scene, and exactly what a context given the edited scene by a full upload renders. Then a
    rotation (apply_rotate: mesh-local rotation + BVH rebuild, re-uploaded) is checked the same way."""
    sc = pt.cornell_scene(pt.torus_knot(80, 24), cube_length=32)  # meshes: 0 walls, 1 light, 2 knot
    cfg = pt.configuration(max_tracer_depth=6)
    cam = pt.camera(64, 40, **BENCH_CAM)
    r, fresh = pt.Renderer(0), pt.Renderer(0)
    try:
        r.upload(sc, cfg)
        r.attach_mesh(sc, 2)
        r.attach_mesh(sc, 1)
        moves = [(2, (0.4, 1.3, -1.2), (0.8, 0.6, 0.7)), (1, (0.2, 2.9, 0.3), (0.6, 0.05, 0.9)),
                 (2, (-0.9, 0.8, -0.4), (0.5, 0.5, 0.5))]
        for mesh, pos, scl in moves:
            r.set_mesh_transform(mesh, pos, scl)
            sc.set_transform(mesh, pos, scl)
            r.setup_frame(64, 40)
            r.render(cam, cfg, 1, 2, write_u8=2)
            img, img8 = r.download()
            ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, 2)
            assert_bitwise(img.reshape(-1, 3), ref, f"refit mesh {mesh} float")
            assert_bitwise(img8.reshape(-1, 3), ref8, f"refit mesh {mesh} 8-bit")
            fresh.upload(sc, cfg)
            fresh.setup_frame(64, 40)
            fresh.render(cam, cfg, 1, 2, write_u8=2)
            assert np.array_equal(fresh.download()[0], img)
        sc.set_rotate(2, (25.0, -40.0, 10.0))
        sc.apply_rotate(2)
        r.upload(sc, cfg)
        img, img8, ref, ref8, _ = render_both(r, sc, cam, cfg, passes=2)
        assert_bitwise(img, ref, "apply_rotate float")
        assert_bitwise(img8, ref8, "apply_rotate 8-bit")
    finally:
        r.close()
        fresh.close()
