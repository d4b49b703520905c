"""Randomised whole-frame parity: seeded random scenes from the reference's building blocks, rendered by the
HIP renderer under both schedules and checked against the oracle bit for bit, float running sum and 8-bit image.

The fixed parity tests each pin one feature on one scene; these cases mix them: 0-4 spheres and 0-3 meshes
(Cornell walls, rotated cubes, torus knots, at leaf size 1 or 3) with materials drawn from the reference
presets (metals, dielectrics, GGX roughness, emissive, scattering and absorbing media, textured diffuse and
specular maps of ragged sizes), configuration switches (anti-aliasing, bilinear filtering, sky box / sky /
black background, gamma, an air medium, the energy threshold, the depth cap including 0), a thin-lens camera,
ragged frame sizes (down to 1 pixel) and a second call that continues the running sum (pass_counter > 1,
path_tracer_kernel.cu:644-651). Every case is its own seed (numpy PCG64), so a failure names a reproducible
scene. Most cases carry an emitter or a sky so that paths return radiance (asserted over the whole set by
test_random_scene_set_is_lit, CPU only).

Reference: Kernel/path_tracer_kernel.cu:275-651 (the radiance loop), Core/material.cpp (presets),
Core/texture.h / Core/cube_map.h (lookups), Bvh/bvh.cpp (leaf sizes).
"""
import numpy as np
import pytest

import oracle
import pathtracerwithcuda_amd as pt

MATERIALS = ["iron", "gold", "silver", "copper", "glass", "green_glass", "diamond", "red", "blue", "wall_white",
             "wall_red", "marble", "something_blue", "something_red", "light", "DragonGreen", "diffuse_white",
             "Micro1", "Micro3", "Micro6"]
CASES = 384


def random_case(seed: int):
    """(scene, configuration, camera, first_pass, pass_count) of case `seed`."""
    rng = np.random.default_rng(seed)
    leaf = int(rng.choice([1, 1, 3]))
    sc = pt.Scene()
    textures = []
    if rng.random() < 0.4:
        for hi in (40, 9):
            h, w = int(rng.integers(1, hi + 1)), int(rng.integers(1, hi + 1))
            textures.append(sc.add_texture(rng.integers(0, 256, (h, w, 4), dtype=np.uint8)))

    def mat():
        name = str(rng.choice(MATERIALS))
        if textures and rng.random() < 0.5:
            ids = textures + [-1]
            return sc.add_material(pt.material(name, diffuse_texture_id=int(rng.choice(ids)),
                                               specular_texture_id=int(rng.choice(ids))))
        return sc.add_material(name)

    for _ in range(int(rng.integers(0, 5))):
        sc.add_sphere(tuple(rng.uniform(-2.0, 2.0, 3)), float(rng.uniform(0.05, 1.2)), str(rng.choice(MATERIALS)))
    for kind in rng.choice(["walls", "cube", "knot"], size=int(rng.integers(0, 4))):
        if kind == "walls":
            sc.add_mesh(pt.cornell_shapes(), [mat() for _ in range(5)], position=(0.0, -0.8, 1.0),
                        scale=(0.1, 0.1, 0.3))
        elif kind == "cube":
            sc.add_mesh([pt.cube_shape()], [mat()], position=tuple(rng.uniform(-1.5, 1.5, 3)),
                        scale=(float(rng.uniform(0.2, 1.5)),) * 3, rotate=tuple(rng.uniform(0.0, 90.0, 3)))
        else:
            knot = pt.torus_knot(int(rng.integers(12, 41)), int(rng.integers(3, 11)))
            sc.add_mesh([knot], [mat()], position=tuple(rng.uniform(-1.0, 1.0, 3)),
                        scale=(float(rng.uniform(0.3, 1.2)),) * 3)
    if rng.random() < 0.6:  # an emitter: a light panel or a light sphere
        if rng.random() < 0.5:
            sc.add_mesh([pt.cube_shape()], [sc.add_material("light")], position=(0.0, 3.1, 0.0),
                        scale=(0.85, 0.05, 0.85))
        else:
            sc.add_sphere(tuple(rng.uniform(-2.0, 2.0, 3)), float(rng.uniform(0.2, 0.8)), "light")
    sky_box = rng.random() < 0.5
    if sky_box:
        sc.set_cube_map(pt.procedural_cube_map(int(rng.choice([1, 2, 8, 16])), seed=seed))
    sc.build(leaf_size=leaf)
    cfg_kw = dict(max_tracer_depth=int(rng.integers(0, 10)), use_anti_alias=int(rng.random() < 0.7),
                  use_bilinear=int(rng.random() < 0.5), use_sky_box=int(sky_box and rng.random() < 0.8),
                  use_sky=int(rng.random() < 0.5), gamma_correction=int(rng.random() < 0.7),
                  energy_exist_threshold=float(rng.choice([0.000001, 0.01, 0.2])), bvh_leaf_node_triangle_num=leaf)
    if rng.random() < 0.3:
        cfg_kw.update(air_absorption_coef=tuple(rng.uniform(0.0, 0.3, 3)),
                      air_reduced_scattering_coef=tuple(rng.uniform(0.0, 0.3, 3)))
    cfg = pt.configuration(**cfg_kw)
    W, H = int(rng.integers(1, 65)), int(rng.integers(1, 49))
    aperture = float(rng.choice([0.0, 0.0, 0.05, 0.3]))
    cam = pt.camera(W, H, fov=float(rng.choice([30.0, 45.0, 80.0])), yaw=float(rng.uniform(-3.1, 3.1)),
                    pitch=float(rng.uniform(-1.2, 1.2)), radius=float(rng.uniform(3.0, 14.0)),
                    aperture=aperture, focal=float(rng.uniform(2.0, 14.0)) if aperture else None)
    return sc, cfg, cam, int(rng.integers(1, 5)), int(rng.integers(1, 6))


def test_random_scene_set_is_lit():
    """CPU: the case set is not trivially black — most cases return radiance in the oracle."""
    lit = 0
    for seed in range(CASES):
        sc, cfg, cam, first, count = random_case(seed)
        try:
            ref, _, _ = oracle.render(sc.view, cam, cfg, 1, first - 1 + count)
            lit += bool(np.nanmax(np.abs(ref)) > 0) if ref.size else 0
        finally:
            sc.close()
    assert lit >= CASES // 2, f"only {lit} of {CASES} random cases return any radiance"


@pytest.fixture(scope="module")
def renderers(require_gpu):
    rs = {}
    for schedule in ("persistent", "wavefront"):
        r = pt.Renderer(0)
        r.set_schedule(schedule)
        rs[schedule] = r
    yield rs
    for r in rs.values():
        r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(CASES))
def test_random_scene_frame_equals_the_oracle(renderers, seed):
    sc, cfg, cam, first, count = random_case(seed)
    try:
        W, H = int(cam.resolution[0]), int(cam.resolution[1])
        # passes 1..first-1, then first..first+count-1 continuing the running sum, against one oracle run of
        # all the passes
        ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, first - 1 + count)
        for schedule, r in renderers.items():
            r.upload(sc, cfg)
            r.setup_frame(W, H)
            if first > 1:
                r.render(cam, cfg, 1, first - 1, write_u8=0)
            r.render(cam, cfg, first, count, write_u8=2)
            r.synchronize()
            img, img8 = r.download()
            a, b = img.reshape(-1, 3), ref.reshape(-1, 3)
            same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
            assert same.all(), (f"seed {seed} {schedule}: {int((~same).any(axis=1).sum())} of {W * H} pixels differ "
                                f"(passes {first}..{first + count - 1}, depth {cfg.max_tracer_depth})")
            assert np.array_equal(img8.reshape(-1, 3), ref8.reshape(-1, 3)), f"seed {seed} {schedule}: 8-bit differs"
    finally:
        sc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(96))
def test_random_scene_frame_groups_equal_the_oracle(renderers, seed):
    """pt_render_frames (the MULTI instances, one per scene feature set) on the same random scenes: 2-5 frames,
    each through its own camera, one launch per batch of passes, with a random band share (rows of one band
    index of 1-3, bands of 1-8 rows) and grid share. Every frame's owned rows against the oracle's frame of its
    camera, bit for bit; rows outside the share keep the caller's fill value."""
    import torch

    sc, cfg, cam0, first, count = random_case(10_000 + seed)
    rng = np.random.default_rng(20_000 + seed)
    try:
        W, H = int(cam0.resolution[0]), int(cam0.resolution[1])
        cams = [cam0] + [pt.camera(W, H, yaw=float(rng.uniform(-3.1, 3.1)), pitch=float(rng.uniform(-1.0, 1.0)),
                                   radius=float(rng.uniform(3.0, 14.0))) for _ in range(int(rng.integers(1, 5)))]
        band_rows, band_count = int(rng.choice([1, 3, 8])), int(rng.integers(1, 4))
        band_index = int(rng.integers(0, band_count))
        r = renderers["persistent"]
        r.upload(sc, cfg)
        r.setup_frame(W, H)
        r.set_tiling(band_rows, band_count, band_index)
        r.set_grid_share(int(rng.choice([100, 100, 45, 10])))
        try:
            n = W * H * 3
            imgs = [torch.full((n,), 7.0, dtype=torch.float32, device="cuda:0") for _ in cams]
            imgs8 = [torch.zeros((n,), dtype=torch.uint8, device="cuda:0") for _ in cams]
            if first > 1:
                r.render_frames(cams, cfg, imgs, imgs8, 1, first - 1, write_u8=0)
            r.render_frames(cams, cfg, imgs, imgs8, first, count, write_u8=2)
            r.synchronize()
        finally:
            r.set_tiling(1, 1, 0)
            r.set_grid_share(100)
        rows = [y for y in range(H) if (y // band_rows) % band_count == band_index]
        other = [y for y in range(H) if y not in rows]
        for f, cam in enumerate(cams):
            ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, first - 1 + count)
            img = imgs[f].cpu().numpy().reshape(H, W, 3)
            a, b = img[rows].reshape(-1, 3), ref.reshape(H, W, 3)[rows].reshape(-1, 3)
            same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
            assert same.all(), f"seed {seed} frame {f}: {int((~same).any(axis=1).sum())} pixels differ"
            assert np.array_equal(imgs8[f].cpu().numpy().reshape(H, W, 3)[rows], ref8.reshape(H, W, 3)[rows])
            assert (img[other] == 7.0).all(), f"seed {seed} frame {f}: rows outside the share written"
    finally:
        sc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(64))
def test_random_scene_medium_bound_equals_the_oracle(renderers, seed):
    """The medium-bounded walk (pt_set_medium_bound, a tolerance mode) on random scenes whose materials and air
    include scattering media: the HIP frame equals the oracle's bounded walk bit for bit (the persistent
    schedule; the wavefront schedule walks exactly)."""
    sc, cfg, cam, first, count = random_case(30_000 + seed)
    rng = np.random.default_rng(40_000 + seed)
    cfg.air_reduced_scattering_coef = pt._abi.Float3(*map(float, rng.uniform(0.0, 2.0, 3)))
    cfg.air_absorption_coef = pt._abi.Float3(*map(float, rng.uniform(0.0, 0.5, 3)))
    r = renderers["persistent"]
    try:
        W, H = int(cam.resolution[0]), int(cam.resolution[1])
        ref, ref8, _ = oracle.render(sc.view, cam, cfg, 1, first - 1 + count, medium_bound=True)
        r.set_medium_bound(True)
        try:
            r.upload(sc, cfg)
            r.setup_frame(W, H)
            if first > 1:
                r.render(cam, cfg, 1, first - 1, write_u8=0)
            r.render(cam, cfg, first, count, write_u8=2)
            r.synchronize()
            img, img8 = r.download()
        finally:
            r.set_medium_bound(False)
        a, b = img.reshape(-1, 3), ref.reshape(-1, 3)
        same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
        assert same.all(), f"seed {seed}: {int((~same).any(axis=1).sum())} of {W * H} pixels differ"
        assert np.array_equal(img8.reshape(-1, 3), ref8.reshape(-1, 3)), f"seed {seed}: 8-bit differs"
    finally:
        sc.close()


def test_random_media_bounded_walk_equals_exact():
    """CPU: on the same 64 random scenes with a scattering air (and whatever media their materials carry), the
    oracle's medium-bounded walk renders every pixel identical to the exact walk — the tolerance mode's measured
    contract on scenes it was not tuned on."""
    differing = []
    for seed in range(64):
        sc, cfg, cam, first, count = random_case(30_000 + seed)
        rng = np.random.default_rng(40_000 + seed)
        cfg.air_reduced_scattering_coef = pt._abi.Float3(*map(float, rng.uniform(0.0, 2.0, 3)))
        cfg.air_absorption_coef = pt._abi.Float3(*map(float, rng.uniform(0.0, 0.5, 3)))
        try:
            a, _, _ = oracle.render(sc.view, cam, cfg, 1, first - 1 + count, medium_bound=True)
            b, _, _ = oracle.render(sc.view, cam, cfg, 1, first - 1 + count)
        finally:
            sc.close()
        a, b = a.reshape(-1, 3), b.reshape(-1, 3)
        same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
        if not same.all():
            differing.append((seed, int((~same).any(axis=1).sum())))
    assert not differing, f"bounded walk differs from the exact walk: {differing}"
