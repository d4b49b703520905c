"""pt_render, the headless C++ host program (csrc/pt_cli.cpp): the reference application's
config -> scene -> camera -> render passes -> screenshot sequence (Main/window.cpp:115-412, 712-740)
without the window. GPU tests compare its PNG with the oracle's 8-bit image of the same scene,
camera and passes, through the native path and through the reference ABI (path_tracer_kernel called
pass by pass as Core/path_tracer.cpp:40-67 does)."""
import json
import os
import subprocess

import numpy as np
import pytest

import pathtracerwithcuda_amd as pt
from pathtracerwithcuda_amd.build import CLI

PIL = pytest.importorskip("PIL.Image")


def run_cli(*args):
    return subprocess.run([CLI, *map(str, args)], capture_output=True, text=True, timeout=300)


def test_cli_usage_and_argument_errors():
    assert os.path.exists(CLI)
    assert run_cli("--help").returncode == 2
    assert run_cli("--width", "8").returncode == 2  # no scene
    assert run_cli("--scene", "x.json", "--bogus", "1").returncode == 2


def test_cli_fails_loudly_on_missing_inputs(tmp_path):
    r = run_cli("--scene", str(tmp_path / "missing.json"))
    assert r.returncode != 0 and "[Error]" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("abi", [False, True])
def test_cli_png_equals_oracle(require_gpu, tmp_path, abi):
    import oracle
    from test_loader import make_root

    root = make_root(tmp_path)
    cfgp = root / "res" / "configuration" / "config.json"
    scene = root / "res" / "scene" / "cornell_box_simple.json"
    out = tmp_path / "o.png"
    W, H, spp, depth = 48, 36, 3, 5
    cam_kw = dict(pitch=0.08, radius=12.5, center=(0.0, 1.2, 0.0))
    args = ["--scene", scene, "--root", root, "--config", cfgp, "--width", W, "--height", H, "--spp", spp,
            "--depth", depth, "--pitch", cam_kw["pitch"], "--radius", cam_kw["radius"], "--center", "0,1.2,0",
            "--out", out]
    if abi:
        args.append("--abi")
    r = run_cli(*args)
    assert r.returncode == 0, r.stderr[-2000:]
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["width"] == W and info["spp"] == spp and info["triangles"] == 22
    got = np.asarray(PIL.open(str(out)).convert("RGB"))

    cfg = pt.load_config(str(cfgp))
    cfg.width, cfg.height, cfg.max_tracer_depth = W, H, depth
    sc = pt.load_scene(str(scene), root_dir=str(root), config=cfg)
    cam = pt.camera(W, H, **cam_kw)
    _, ref8, _ = oracle.render(sc.view, cam, cfg, 1, spp)
    assert np.array_equal(got.reshape(-1, 3), ref8)
