"""Headless image output (the reference's only output is an interactive PNG screenshot,
Main/window.cpp:712-740, via lodepng): 8-bit PNG of the uchar3 image and PFM of the float3
running sum. Row 0 of the renderer's buffers is the top of the image.

PNG encoding and decoding are the C++ ones of libpt_hip.so (csrc/pt_image.cpp, pinned against the
reference's vendored lodepng in tests/test_ref_pin.py); this module only adapts array shapes."""
from __future__ import annotations

import numpy as np

from .loader import load_image
from .loader import write_png as _write_png


def write_png(path: str, rgb8: np.ndarray) -> None:
    """(H, W, 3) or (H, W, 4) uint8, top row first -> PNG (pt_image_write_png)."""
    _write_png(path, np.ascontiguousarray(rgb8, np.uint8))


def read_png_rgb(path: str) -> np.ndarray:
    """PNG -> (H, W, 3) uint8, top row first (pt_image_load)."""
    return load_image(path)[:, :, :3]


def write_pfm(path: str, rgb: np.ndarray) -> None:
    """PFM is bottom row first; flip so the file shows the same picture as the PNG."""
    rgb = np.ascontiguousarray(rgb[::-1], "<f4")
    h, w, _ = rgb.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(rgb.tobytes())


def screenshot_name(frame_ms: float, spp: int, render_s: float, width: int, height: int) -> str:
    """Main/window.cpp:728 naming: FrameTime-%dms_SSP-%d_RenderTime-%ds_%dX%d.png"""
    return f"FrameTime-{int(frame_ms)}ms_SSP-{spp}_RenderTime-{int(render_s)}s_{width}X{height}.png"
