"""The host ingestion layer under AddressSanitizer + UndefinedBehaviorSanitizer: the
hand-written JSON, OBJ, BMP/TGA/PNG (zlib-fed) parsers and the BVH builders (pt_loader.cpp, pt_image.cpp,
pt_host.cpp), linked into tools/san/san_driver with -fsanitize=address,undefined, run over the
reference's own fixtures (tests/golden/res) and over truncated and bit-flipped copies of every file.
Loaders may reject corrupted input (that is their error path); a sanitizer report or a crash fails."""
import fcntl
import os
import subprocess

import numpy as np
import pytest

from test_loader import RES, make_root

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(os.path.dirname(HERE), "tools", "san")
DRIVER = os.path.join(SAN, "build", "san_driver")
PIL = pytest.importorskip("PIL.Image")


@pytest.fixture(scope="module")
def driver():
    # one build at a time when pytest-xdist workers share the tree (make relinks a running driver otherwise)
    os.makedirs(os.path.join(SAN, "build"), exist_ok=True)
    with open(os.path.join(SAN, "build", ".lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", SAN], check=True, capture_output=True)
    return DRIVER


def run(driver, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=97",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")
    env.pop("LD_PRELOAD", None)
    res = subprocess.run([driver, *map(str, args)], capture_output=True, text=True, timeout=600, env=env)
    report = res.stderr
    assert res.returncode == 0, f"{args[:2]} exit {res.returncode}\n{report[-3000:]}"
    assert "AddressSanitizer" not in report and "runtime error" not in report, report[-3000:]
    return res.stdout


def corrupt_copies(src, out_dir, seeds=4):
    """Truncations at several lengths and random byte flips of one file."""
    data = open(src, "rb").read()
    base = os.path.basename(src)
    paths = []
    for frac in (0.0, 0.01, 0.1, 0.5, 0.9, 0.999):
        p = os.path.join(out_dir, f"trunc{frac}_{base}")
        open(p, "wb").write(data[:int(len(data) * frac)])
        paths.append(p)
    rng = np.random.default_rng(len(data))
    for s in range(seeds):
        b = bytearray(data)
        if b:
            for i in rng.integers(0, len(b), max(1, len(b) // 200)):
                b[i] = int(rng.integers(0, 256))
        p = os.path.join(out_dir, f"flip{s}_{base}")
        open(p, "wb").write(bytes(b))
        paths.append(p)
    return paths


def test_config_and_obj_parsers(driver, tmp_path):
    cfgs = [os.path.join(RES, "configuration", "config.json")]
    objs = [os.path.join(RES, "obj", f) for f in sorted(os.listdir(os.path.join(RES, "obj")))]
    bad = []
    for f in cfgs + objs:
        bad += corrupt_copies(f, str(tmp_path))
    out = run(driver, "config", *cfgs, *[p for p in bad if p.endswith(".json")])
    assert "config.json: 0" in out
    out = run(driver, "obj", *objs, *[p for p in bad if p.endswith(".obj")])
    assert "cornell.obj: 0 (10 triangles)" in out


def _images(d):
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, (19, 23, 3), dtype=np.uint8)
    rgba = rng.integers(0, 256, (17, 31, 4), dtype=np.uint8)
    paths = []
    for name, img, kw in (("rgb.png", PIL.fromarray(rgb, "RGB"), {}),
                          ("rgba_interlaced.png", PIL.fromarray(rgba, "RGBA"), {"interlace": 1}),
                          ("pal.png", PIL.fromarray(rgb, "RGB").quantize(16), {}),
                          ("gray16.png", PIL.fromarray(rgb[..., 0].astype(np.uint16) * 257), {}),
                          ("rgb.bmp", PIL.fromarray(rgb, "RGB"), {}),
                          ("pal.bmp", PIL.fromarray(rgb, "RGB").quantize(16), {}),
                          ("rgb.tga", PIL.fromarray(rgb, "RGB"), {}),
                          ("rgba_rle.tga", PIL.fromarray(rgba, "RGBA"), {"compression": "tga_rle"}),
                          ("rgb420.jpg", PIL.fromarray(rgb, "RGB"), {"quality": 80, "subsampling": 2}),
                          ("rgb444_rst.jpg", PIL.fromarray(rgb, "RGB"),
                           {"quality": 95, "subsampling": 0, "restart_marker_blocks": 2}),
                          ("grey.jpg", PIL.fromarray(rgb[..., 0], "L"), {"quality": 50}),
                          ("prog.jpg", PIL.fromarray(rgb, "RGB"), {"quality": 70, "progressive": True}),
                          ("prog_rst.jpg", PIL.fromarray(rgb, "RGB"),
                           {"quality": 90, "progressive": True, "restart_marker_blocks": 3})):
        p = os.path.join(d, name)
        img.save(p, **kw)
        paths.append(p)
    return paths


def test_image_decoders_and_png_writer(driver, tmp_path):
    good = _images(str(tmp_path))
    bad = []
    for f in good:
        bad += corrupt_copies(f, str(tmp_path), seeds=6)
    out = run(driver, "image", tmp_path / "out.png", *good, *bad)
    for f in good:
        assert f"{f}: 0 (" in out, out


@pytest.mark.parametrize("name", ["cornell_box_simple", "depth_of_view", "fresnel", "micro_surface",
                                  "refractive_index", "tex_cube"])
def test_scene_loader_and_bvh_builders(driver, tmp_path, name):
    root = make_root(tmp_path)
    scene = root / "res" / "scene" / f"{name}.json"
    args = [root, scene]
    out = run(driver, "scene", *args)
    assert out.count(": rc") == 0, out  # every builder, leaf sizes 1 and 3
    for p in corrupt_copies(str(scene), str(tmp_path)):
        run(driver, "scene", root, p, *args[2:])


@pytest.mark.parametrize("name", ["vanille", "vanille_nude", "subsurface_scattering_s", "dinosaur",
                                  "c5_vanille_gallery"])
def test_scene_loader_on_reference_assets(driver, tmp_path, name):
    """The reference's own larger assets (tests/golden/ref_assets.tar.xz: vanille's 15-shape OBJ and 1024^2 TGA maps,
    the cups, the sponza RGBA/RGB specular maps, the lobby BMP faces) through the loader and every builder under
    ASan/UBSan, with the background override the GPU tests use."""
    root = make_root(tmp_path, assets=True)
    out = run(driver, "scene", root, root / "res" / "scene" / f"{name}.json", "res\\texture\\lobby", "bmp")
    assert out.count(": rc") == 0, out


def test_bvh_builders_on_degenerate_triangles(driver):
    for seed in (1, 2, 3):
        run(driver, "bvh", seed)
