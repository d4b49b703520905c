#!/usr/bin/env python3
"""Packs the reference's own asset files that the GPU tests and `bench.py --workload c5` render into
tests/golden/ref_assets.tar.xz (data fixtures: meshes, textures, skybox faces — no source). The pack is git-ignored
(the reference states no license for these assets, and the sponza maps carry their own): __graft_entry__.build()
regenerates it from the checkout; tests that need it skip where it is absent.

/root/reference does not exist on the GPU box, so the scenes that use these assets can only run there
from a committed copy. The pack keeps the reference's directory layout (res/obj, res/texture/...), so
`bench.asset_root()` unpacks it next to tests/golden/res and the reference's scene JSONs load unchanged.

    python tools/pack_ref_assets.py            # rewrites tests/golden/ref_assets.tar.xz
"""
import hashlib
import io
import os
import sys
import tarfile

REF = "/root/reference/gpu_path_tracer"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "ref_assets.tar.xz")

FILES = [
    # meshes of vanille.json, vanille_nude.json, subsurface_scattering_{s,a}.json, dinosaur.json and C5
    "res/obj/vanille.obj", "res/obj/vanille_nude.obj", "res/obj/cup.obj", "res/obj/dinosaur.obj",
    "res/obj/human.obj", "res/obj/cow.obj", "res/obj/monkey.obj",
    # vanille.json's five diffuse maps, vanille_nude.json's two present maps (c595_00.tga is missing upstream)
    "res/texture/vanille/c005_16.tga", "res/texture/vanille/c005_09.tga", "res/texture/vanille/c005_05.tga",
    "res/texture/vanille/c005_03.tga", "res/texture/vanille/c005_10.tga",
    "res/texture/vanille_nude/c595_03.tga", "res/texture/vanille_nude/c595_05.tga",
    # C5's specular maps (sponza *_spec.tga): 512^2 RGBA, 512^2 RGB, 1024^2 RGB
    "res/texture/sponza/spnza_bricks_a_spec.tga", "res/texture/sponza/sponza_thorn_spec.tga",
    "res/texture/sponza/sponza_column_a_spec.tga",
    # the lobby skybox (512^2 BMP faces): the background of every scene whose own skybox is missing or JPEG
    *[f"res/texture/lobby/{f}.bmp" for f in ("xpos", "xneg", "ypos", "yneg", "zpos", "zneg")],
]


def main() -> int:
    if not os.path.isdir(REF):
        print("the reference checkout is absent", file=sys.stderr)
        return 1
    buf = io.BytesIO()
    # deterministic archive: sorted names, fixed mtime/owner, so the pack only changes when the files do
    with tarfile.open(fileobj=buf, mode="w:xz", preset=9) as tar:
        for rel in sorted(FILES):
            data = open(os.path.join(REF, rel), "rb").read()
            info = tarfile.TarInfo(rel)
            info.size = len(data)
            info.mtime = 0
            info.mode = 0o444
            tar.addfile(info, io.BytesIO(data))
    if os.path.exists(OUT) and open(OUT, "rb").read() == buf.getvalue():
        print(f"{OUT}: unchanged")
        return 0
    open(OUT, "wb").write(buf.getvalue())
    print(f"{OUT}: {len(FILES)} files, {len(buf.getvalue())} bytes, sha256 {hashlib.sha256(buf.getvalue()).hexdigest()[:16]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
