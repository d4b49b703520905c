"""JPEG decoding (pt_jpeg.cpp) for the reference's JPEG skyboxes (res/scene/*.json "Format": "jpg",
loaded through FreeImage_Load with flags 0: Others/image_loader.cpp:31-95).

FreeImage's default JPEG load is libjpeg's fast integer IDCT without fancy upsampling (FreeImage.h:693).
PIL's decoder runs libjpeg-turbo in that same mode when its draft flag is set. libjpeg-turbo keeps
libjpeg 6b's arithmetic, so the decoder's 6b variant must equal PIL bit for bit. That pins the parts
both variants share: markers, Huffman decoding, dequantisation, block layout, upsampling and colour
conversion. The 9a variant (what the reference's FreeImage 3.17 ran, and what pt_image_load uses)
differs from 6b only in the IDCT's rounding and the colour coefficients. Those lines are restated
from libjpeg 9a and unpinned."""
import glob
import io
import os

import numpy as np
import pytest

import pathtracerwithcuda_amd as pt
from pathtracerwithcuda_amd import loader

PIL = pytest.importorskip("PIL.Image")
REF_TEX = "/root/reference/gpu_path_tracer/res/texture"


def pil_fast(data: bytes) -> np.ndarray:
    """libjpeg-turbo with the fast IDCT and no fancy upsampling (PIL's draft decoder flag)."""
    im = PIL.open(io.BytesIO(data))
    im.decoderconfig = (1, 1)  # (scale, draft)
    im.load()
    return np.asarray(im.convert("RGB"))


def encode(img, **kw) -> bytes:
    b = io.BytesIO()
    img.save(b, "JPEG", **kw)
    return b.getvalue()


def cases():
    rng = np.random.default_rng(11)
    # smooth gradients plus noise: real-image-like blocks with both small and large coefficients
    y, x = np.mgrid[0:61, 0:77]
    smooth = np.stack([(x * 3) % 256, (y * 4) % 256, ((x + y) * 2) % 256], -1)
    noisy = np.clip(smooth + rng.integers(-40, 41, smooth.shape), 0, 255).astype(np.uint8)
    rgb = PIL.fromarray(noisy, "RGB")
    out = []
    for sub in (0, 1, 2):  # 4:4:4, 4:2:2, 4:2:0
        for q in (30, 75, 95):
            out.append((f"sub{sub}_q{q}", encode(rgb, quality=q, subsampling=sub)))
    out.append(("optimized", encode(rgb, quality=80, optimize=True)))
    out.append(("restart_blocks", encode(rgb, quality=85, subsampling=2, restart_marker_blocks=3)))
    out.append(("restart_rows", encode(rgb, quality=60, subsampling=1, restart_marker_rows=1)))
    out.append(("grey", encode(PIL.fromarray(noisy[..., 1], "L"), quality=70)))
    out.append(("tiny", encode(PIL.fromarray(noisy[:5, :3], "RGB"), quality=90)))
    out.append(("q100_444", encode(rgb, quality=100, subsampling=0)))
    # progressive (SOF2): spectral selection and successive approximation scans, end-of-band runs
    for sub in (0, 2):
        out.append((f"prog_sub{sub}", encode(rgb, quality=80, subsampling=sub, progressive=True)))
    out.append(("prog_optimized", encode(rgb, quality=40, progressive=True, optimize=True)))
    out.append(("prog_restart", encode(rgb, quality=90, progressive=True, restart_marker_blocks=5)))
    out.append(("prog_grey", encode(PIL.fromarray(noisy[..., 2], "L"), quality=85, progressive=True)))
    flat = np.zeros((40, 48, 3), np.uint8)
    flat[8:30, 10:40] = (200, 40, 90)  # long end-of-band runs
    out.append(("prog_flat", encode(PIL.fromarray(flat, "RGB"), quality=75, progressive=True)))
    return out


@pytest.mark.parametrize("name,data", cases(), ids=[c[0] for c in cases()])
def test_ijg6_variant_equals_libjpeg_turbo_fast_mode(name, data):
    got = loader.decode_jpeg(data, loader.JPEG_IJG6)
    want = pil_fast(data)
    assert got.shape[:2] == want.shape[:2]
    assert np.array_equal(got[..., :3], want), f"{np.count_nonzero(got[..., :3] != want)} samples differ"
    assert (got[..., 3] == 255).all()


@pytest.mark.parametrize("name,data", cases()[:4], ids=[c[0] for c in cases()[:4]])
def test_ijg9_variant_differs_only_by_rounding(name, data):
    a9 = loader.decode_jpeg(data, loader.JPEG_IJG9)[..., :3].astype(int)
    a6 = loader.decode_jpeg(data, loader.JPEG_IJG6)[..., :3].astype(int)
    d = np.abs(a9 - a6)
    # per sample: the IDCT's final rounding (<= 1 per component), the odd part's floor of a negated
    # product, and the colour tables' coefficients; a few levels at most after colour conversion
    assert d.max() <= 3 and d.any()


def test_load_image_decodes_jpeg_as_libjpeg_9a(tmp_path):
    data = cases()[5][1]
    p = tmp_path / "face.jpg"
    p.write_bytes(data)
    assert np.array_equal(pt.load_image(str(p)), loader.decode_jpeg(data, loader.JPEG_IJG9))


def test_unsupported_jpegs_fail_loudly(tmp_path):
    rgb = PIL.fromarray(np.zeros((16, 16, 3), np.uint8), "RGB")
    data = bytearray(encode(rgb))
    i = data.index(b"\xff\xc0")
    data[i + 1] = 0xC9  # the same frame marked arithmetic-coded
    p = tmp_path / "arith.jpg"
    p.write_bytes(bytes(data))
    with pytest.raises(pt.PtError):
        pt.load_image(str(p))
    p = tmp_path / "cmyk.jpg"
    PIL.fromarray(np.zeros((8, 8, 4), np.uint8), "CMYK").save(str(p))
    with pytest.raises(pt.PtError):
        pt.load_image(str(p))
    with pytest.raises(pt.PtError):
        loader.decode_jpeg(b"\xff\xd8\xff\xd9")


@pytest.mark.skipif(not os.path.isdir(REF_TEX), reason="reference checkout not present")
def test_reference_skybox_faces():
    """The reference's own JPEG skyboxes (2048x2048 baseline 4:2:0, lycksele and maskonaive)."""
    faces = sorted(glob.glob(os.path.join(REF_TEX, "**", "*.jpg"), recursive=True))
    assert len(faces) == 12
    for f in faces[::3]:
        data = open(f, "rb").read()
        a6 = loader.decode_jpeg(data, loader.JPEG_IJG6)[..., :3]
        assert np.array_equal(a6, pil_fast(data)), f
        a9 = loader.decode_jpeg(data, loader.JPEG_IJG9)[..., :3].astype(int)
        assert np.abs(a9 - a6.astype(int)).max() <= 3, f
