"""Python face of the C++ ingestion layer (include/pt_loader.h): the reference's config.json and
scene JSON loaders, its OBJ loader and image decoding, as a reference user drives them.

    cfg = load_config("res/configuration/config.json")            # config_parser::load_config
    scene = load_scene("res/scene/cube.json", root_dir=".", config=cfg)   # scene_parser::load_scene
                                                                   #   + create_scene_data_device
Reference: Core/config_parser.cpp:8-187, Core/scene_parser.cpp:37-528, Core/triangle_mesh.cpp:8-213,
Others/image_loader.cpp:31-95.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import Configuration, Material, lib
from .scene import Scene, Shape


def load_config(path: str) -> Configuration:
    """config.json -> reference `configuration` (string-valued keys; FOV parsed as a bool like the
    reference, config_parser.cpp:111). Raises PtError when the file is missing a key or malformed."""
    cfg = Configuration()
    rc = lib().pt_config_load(path.encode(), C.byref(cfg))
    if rc != 0:
        raise _abi.PtError(f"load_config({path!r}) failed ({rc})")
    return cfg


def material_preset(name: str) -> Material:
    """A built-in material (Core/material.cpp:12-577) by its scene-file name."""
    m = Material()
    if lib().pt_material_preset(name.encode(), C.byref(m)) != 0:
        raise KeyError(name)
    return m


def load_obj(path: str) -> list[Shape]:
    """Triangulated OBJ shapes (tinyobjloader 1.1.0 semantics, normals required)."""
    om = _abi.ObjMesh()
    rc = lib().pt_obj_load(path.encode(), C.byref(om))
    if rc != 0:
        raise _abi.PtError(f"load_obj({path!r}) failed ({rc})")
    try:
        n = om.triangle_num
        v = np.ctypeslib.as_array(om.vertices, (n * 9,)).reshape(n, 3, 3).copy() if n else np.zeros((0, 3, 3), np.float32)
        nr = np.ctypeslib.as_array(om.normals, (n * 9,)).reshape(n, 3, 3).copy() if n else np.zeros((0, 3, 3), np.float32)
        uv = (np.ctypeslib.as_array(om.uvs, (n * 6,)).reshape(n, 3, 2).copy() if (n and om.uvs) else None)
        sh = np.ctypeslib.as_array(om.shape_of_triangle, (n,)).copy() if n else np.zeros(0, np.int32)
        shapes = []
        for s in range(om.shape_num):
            sel = sh == s
            shapes.append(Shape(v[sel], nr[sel], uv[sel] if uv is not None else None))
        return shapes
    finally:
        lib().pt_obj_free(C.byref(om))


def load_image(path: str) -> np.ndarray:
    """(H, W, 4) uint8 RGBA, top row first, alpha 255 (FreeImage_ConvertTo24Bits then RGBA)."""
    w, h = C.c_int(), C.c_int()
    px = _abi.c_ubyte_p()
    rc = lib().pt_image_load(path.encode(), C.byref(w), C.byref(h), C.byref(px))
    if rc != 0:
        raise _abi.PtError(f"load_image({path!r}) failed ({rc})")
    try:
        return np.ctypeslib.as_array(px, (h.value, w.value, 4)).copy()
    finally:
        lib().pt_image_free(px)


JPEG_IJG9, JPEG_IJG6 = 0, 1  # include/pt_loader.h PT_JPEG_IJG9 / PT_JPEG_IJG6


def decode_jpeg(data: bytes, variant: int = JPEG_IJG9) -> np.ndarray:
    """JPEG bytes -> (H, W, 4) uint8 RGBA with a chosen libjpeg arithmetic (pt_jpeg_decode): JPEG_IJG9 is
    what load_image uses (FreeImage's libjpeg 9a), JPEG_IJG6 the libjpeg-turbo arithmetic the tests pin."""
    w, h = C.c_int(), C.c_int()
    px = _abi.c_ubyte_p()
    buf = (C.c_ubyte * len(data)).from_buffer_copy(data)
    rc = lib().pt_jpeg_decode(buf, len(data), variant, C.byref(w), C.byref(h), C.byref(px))
    if rc != 0:
        raise _abi.PtError(f"decode_jpeg failed ({rc})")
    try:
        return np.ctypeslib.as_array(px, (h.value, w.value, 4)).copy()
    finally:
        lib().pt_image_free(px)


def write_png(path: str, pixels: np.ndarray) -> None:
    """8-bit RGB or RGBA (H, W, 3|4), top row first, through the C++ writer."""
    pixels = np.ascontiguousarray(pixels, np.uint8)
    h, w, ch = pixels.shape
    rc = lib().pt_image_write_png(path.encode(), w, h, pixels.ctypes.data_as(_abi.c_ubyte_p), ch)
    if rc != 0:
        raise _abi.PtError(f"write_png({path!r}) failed ({rc})")


def load_scene(path: str, root_dir: str | None = None, config: Configuration | None = None,
               background: str | None = None, background_format: str | None = None) -> Scene:
    """A reference scene JSON, loaded and built (one BVH per mesh with the configuration's
    BvhLeafNodeTriangleNum / BvhBuildMethod / BvhBucketMaxDivideInternalNum). Asset paths are
    relative to `root_dir` (the reference's working directory). `background` replaces the
    Background folder (Path + Name) for scenes whose skybox is not in the checkout."""
    opt = _abi.SceneLoadOptions()
    keep = []  # keep the encoded strings alive for the call

    def cstr(s):
        if s is None:
            return None
        b = s.encode()
        keep.append(b)
        return b

    opt.root_dir = cstr(root_dir)
    opt.background_override = cstr(background)
    opt.background_format = cstr(background_format)
    opt.leaf_size = config.bvh_leaf_node_triangle_num if config is not None else 1
    opt.bvh_method = config.bvh_build if config is not None else 2
    opt.bucket_num = config.bvh_bucket_max_divide_internal_num if config is not None else 12
    sc = Scene()
    rc = lib().pt_scene_load(sc._b, path.encode(), C.byref(opt))
    if rc != 0:
        sc.close()
        raise _abi.PtError(f"load_scene({path!r}) failed ({rc})")
    v = _abi.SceneView()
    _abi.check(lib().pt_scene_builder_view(sc._b, C.byref(v)), "scene view")
    sc._view = v
    sc.triangle_count = v.triangle_num
    sc.material_names = [f"m{i}" for i in range(v.material_num)]
    return sc
