"""Headless image output (the reference's only output is an interactive PNG screenshot,
Main/window.cpp:712-740, via lodepng): 8-bit PNG of the uchar3 image and PFM of the float3
running sum. Row 0 of the renderer's buffers is the top of the image."""
from __future__ import annotations

import struct
import zlib

import numpy as np


def write_png(path: str, rgb8: np.ndarray) -> None:
    rgb8 = np.ascontiguousarray(rgb8, np.uint8)
    h, w, _ = rgb8.shape
    raw = b"".join(b"\x00" + rgb8[y].tobytes() for y in range(h))

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


def read_png_rgb(path: str) -> np.ndarray:
    """Minimal reader for the 8-bit RGB/RGBA, non-interlaced PNGs this module writes."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w = 8, b"", 0
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        tag = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert depth == 8 and ctype in (2, 6)
            ch = 3 if ctype == 2 else 4
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    stride = w * ch
    out = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = np.frombuffer(raw, np.uint8, stride, y * (stride + 1) + 1).astype(np.int32)
        if f == 0:
            cur = line
        elif f == 2:
            cur = (line + prev) & 255
        else:  # filters 1/3/4 need per-pixel recurrences
            cur = np.zeros(stride, np.int32)
            for x in range(stride):
                a = cur[x - ch] if x >= ch else 0
                b = prev[x]
                c = prev[x - ch] if x >= ch else 0
                if f == 1:
                    cur[x] = (line[x] + a) & 255
                elif f == 3:
                    cur[x] = (line[x] + (a + b) // 2) & 255
                else:
                    p = a + b - c
                    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                    pr = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
                    cur[x] = (line[x] + pr) & 255
        out[y] = cur
        prev = cur
    return out.reshape(h, w, ch)[:, :, :3]


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
