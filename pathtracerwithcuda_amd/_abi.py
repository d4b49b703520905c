"""ctypes mirror of include/pt_types.h, include/pt_host.h, include/pt_native.h and
include/path_tracer_kernel.h, plus the loader for libpt_hip.so.

The library is the product: when it is missing or fails to load, every entry point raises — there
is no CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes as C
import os

from .build import LIB

c_float_p = C.POINTER(C.c_float)
c_int_p = C.POINTER(C.c_int)
c_ubyte_p = C.POINTER(C.c_ubyte)


class Float3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Float2(C.Structure):
    _pack_ = 8
    _fields_ = [("x", C.c_float), ("y", C.c_float)]


class UChar3(C.Structure):
    _fields_ = [("x", C.c_ubyte), ("y", C.c_ubyte), ("z", C.c_ubyte)]


class Ray(C.Structure):  # Core/ray.h:9-18
    _fields_ = [("origin", Float3), ("direction", Float3)]


class Scattering(C.Structure):  # Core/material.h:17-29
    _fields_ = [("absorption_coefficient", Float3), ("reduced_scattering_coefficient", Float3)]


class Medium(C.Structure):  # Core/material.h:31-47
    _fields_ = [("refraction_index", C.c_float), ("extinction_coefficient", C.c_float), ("scattering", Scattering)]


class Material(C.Structure):  # Core/material.h:49-78
    _fields_ = [
        ("diffuse_color", Float3),
        ("emission_color", Float3),
        ("specular_color", Float3),
        ("is_transparent", C.c_ubyte),
        ("roughness", C.c_float),
        ("medium", Medium),
        ("diffuse_texture_id", C.c_int),
        ("specular_texture_id", C.c_int),
    ]


class Sphere(C.Structure):  # Core/sphere.h:11-16
    _fields_ = [("center", Float3), ("radius", C.c_float), ("mat", Material)]


class Triangle(C.Structure):  # Core/triangle.h:10-25
    _fields_ = [
        ("vertex0", Float3), ("vertex1", Float3), ("vertex2", Float3),
        ("normal0", Float3), ("normal1", Float3), ("normal2", Float3),
        ("uv0", C.c_float * 2), ("uv1", C.c_float * 2), ("uv2", C.c_float * 2),
        ("mat", C.POINTER(Material)),
    ]


class BoundingBox(C.Structure):  # Bvh/bounding_box.h:7-10
    _fields_ = [("left_bottom", Float3), ("right_top", Float3), ("centroid", Float3)]


class BvhNodeDevice(C.Structure):  # Bvh/bvh_node.h:41-47
    _fields_ = [
        ("box", BoundingBox),
        ("_pad", C.c_uint32),
        ("triangle_indices", c_int_p),
        ("is_leaf", C.c_ubyte),
        ("next_node_index", C.c_int),
    ]


class BvhNodeMorton(C.Structure):  # Bvh/bvh_node.h:27-39 (bvh_node_morton_code_cuda)
    _fields_ = [
        ("box", BoundingBox), ("left_index", C.c_int), ("right_index", C.c_int), ("parent_index", C.c_int),
        ("is_left_leaf", C.c_ubyte), ("is_right_leaf", C.c_ubyte), ("is_leaf", C.c_ubyte),
        ("triangle_index", C.c_int), ("morton_code", C.c_uint), ("is_visited", C.c_int),
    ]


class RenderCamera(C.Structure):  # Core/camera.h:14-23
    _fields_ = [
        ("eye", Float3), ("view", Float3), ("up", Float3), ("_pad", C.c_uint32),
        ("resolution", C.c_float * 2), ("fov", C.c_float * 2),
        ("aperture_radius", C.c_float), ("focal_distance", C.c_float),
    ]


class Configuration(C.Structure):  # Core/configuration.h:9-34
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int), ("use_fullscreen", C.c_ubyte),
        ("block_size", C.c_int), ("max_block_size", C.c_int), ("max_tracer_depth", C.c_int),
        ("vector_bias_length", C.c_float), ("energy_exist_threshold", C.c_float), ("sss_threshold", C.c_float),
        ("use_sky_box", C.c_ubyte), ("use_sky", C.c_ubyte), ("use_bilinear", C.c_ubyte),
        ("gamma_correction", C.c_ubyte), ("use_anti_alias", C.c_ubyte),
        ("fov", C.c_float), ("bvh_leaf_node_triangle_num", C.c_int), ("bvh_bucket_max_divide_internal_num", C.c_int),
        ("bvh_build_block_size", C.c_int), ("bvh_build", C.c_int), ("air_refraction_index", C.c_float),
        ("air_absorption_coef", Float3), ("air_reduced_scattering_coef", Float3), ("cuda_acceleration", C.c_ubyte),
    ]


class CubeMap(C.Structure):  # Core/cube_map.h:9-18
    _fields_ = [
        ("m_x_positive_map", c_ubyte_p), ("m_x_negative_map", c_ubyte_p),
        ("m_y_positive_map", c_ubyte_p), ("m_y_negative_map", c_ubyte_p),
        ("m_z_positive_map", c_ubyte_p), ("m_z_negative_map", c_ubyte_p),
        ("length", C.c_int),
    ]


class TextureWrapper(C.Structure):  # Core/texture.h:9-13
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("pixels", c_ubyte_p)]


class SceneView(C.Structure):  # include/pt_host.h
    _fields_ = [
        ("mesh_num", C.c_int),
        ("bvh_nodes", C.POINTER(C.POINTER(BvhNodeDevice))),
        ("triangles", C.POINTER(Triangle)),
        ("triangle_num", C.c_int),
        ("sphere_num", C.c_int),
        ("spheres", C.POINTER(Sphere)),
        ("sky_cube_map", C.POINTER(CubeMap)),
        ("mesh_textures", C.POINTER(TextureWrapper)),
        ("texture_num", C.c_int),
        ("materials", C.POINTER(Material)),
        ("material_num", C.c_int),
        ("mesh_node_num", c_int_p),
        ("mesh_triangle_start", c_int_p),
        ("mesh_triangle_num", c_int_p),
    ]


class ViewCamera(C.Structure):  # include/pt_host.h (Core/camera.h:27-80)
    _fields_ = [
        ("center", Float3), ("yaw", C.c_float), ("pitch", C.c_float), ("radius", C.c_float),
        ("aperture_radius", C.c_float), ("focal_distance", C.c_float),
        ("resolution", C.c_float * 2), ("fov", C.c_float * 2),
    ]


class ObjMesh(C.Structure):  # include/pt_loader.h
    _fields_ = [
        ("triangle_num", C.c_int), ("shape_num", C.c_int), ("vertex_num", C.c_int),
        ("vertices", c_float_p), ("normals", c_float_p), ("uvs", c_float_p), ("shape_of_triangle", c_int_p),
    ]


class SceneLoadOptions(C.Structure):  # include/pt_loader.h
    _fields_ = [
        ("root_dir", C.c_char_p), ("background_override", C.c_char_p), ("background_format", C.c_char_p),
        ("leaf_size", C.c_int), ("bvh_method", C.c_int), ("bucket_num", C.c_int),
    ]


LAYOUT = {  # include/pt_types.h static asserts
    "Ray": 24, "Scattering": 24, "Medium": 32, "Material": 84, "Sphere": 100, "Triangle": 104,
    "BoundingBox": 36, "BvhNodeDevice": 56, "BvhNodeMorton": 64, "RenderCamera": 64, "Configuration": 96, "CubeMap": 56,
    "TextureWrapper": 16,
}

# name -> (restype, argtypes)
_PROTOS = {
    # reference ABI (include/path_tracer_kernel.h)
    "path_tracer_kernel": (None, [C.c_int, C.POINTER(C.POINTER(BvhNodeDevice)), C.POINTER(Triangle), C.c_int,
                                  C.POINTER(Sphere), C.c_int, C.POINTER(Float3), C.POINTER(UChar3), C.c_int,
                                  C.POINTER(RenderCamera), C.POINTER(CubeMap), C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.POINTER(TextureWrapper), C.POINTER(Configuration)]),
    "path_tracer_kernel_memory_allocate": (None, [C.POINTER(C.c_void_p)] * 5 + [C.c_int]),
    "path_tracer_kernel_memory_free": (None, [C.c_void_p] * 5),
    "thread_shrink": (C.c_int, [C.c_void_p, C.c_int]),
    # native (include/pt_native.h)
    "pt_last_error": (C.c_char_p, []),
    "pt_sqrt_le_bound": (C.c_float, [C.c_float]),
    "pt_device_count": (C.c_int, []),
    "pt_context_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "pt_context_destroy": (None, [C.c_void_p]),
    "pt_scene_upload": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.POINTER(BvhNodeDevice)), C.POINTER(Triangle),
                                  C.c_int, C.c_int, C.POINTER(Sphere), C.POINTER(CubeMap), C.POINTER(TextureWrapper),
                                  C.c_int, C.POINTER(Configuration)]),
    "pt_scene_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_longlong), c_int_p, c_int_p]),
    "pt_set_grid_share": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_set_medium_bound": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_band_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "pt_set_band_order": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.c_int]),
    "pt_band_cost_enable": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_band_cost": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint), C.c_int]),
    "pt_last_kernel": (C.c_char_p, [C.c_void_p]),
    "pt_mesh_attach": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(Triangle), C.c_int, C.c_int, C.POINTER(BoundingBox),
                                 C.c_int, Float3, Float3]),
    "pt_mesh_set_transform": (C.c_int, [C.c_void_p, C.c_int, Float3, Float3]),
    "pt_frame_setup": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "pt_set_tiling": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int]),
    "pt_render_passes": (C.c_int, [C.c_void_p, C.POINTER(RenderCamera), C.POINTER(Configuration), C.c_int, C.c_int,
                                   C.c_int]),
    "pt_render_frames": (C.c_int, [C.c_void_p, C.POINTER(RenderCamera), C.c_int, C.POINTER(Configuration), C.c_int,
                                   C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "pt_finalize_u8": (C.c_int, [C.c_void_p, C.POINTER(Configuration), C.c_int]),
    "pt_finalize_u8_image": (C.c_int, [C.c_void_p, C.POINTER(Configuration), C.c_int, C.c_void_p, C.c_void_p]),
    "pt_synchronize": (C.c_int, [C.c_void_p]),
    "pt_stream_handle": (C.c_void_p, [C.c_void_p]),
    "pt_image_download": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "pt_image_device_ptr": (C.c_void_p, [C.c_void_p]),
    "pt_image256_device_ptr": (C.c_void_p, [C.c_void_p]),
    "pt_stats_reset": (C.c_int, [C.c_void_p]),
    "pt_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]),
    "pt_stats_all": (C.c_int, [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]),
    "pt_set_instrumented":(C.c_int, [C.c_void_p, C.c_int]),
    "pt_set_schedule":    (C.c_int, [C.c_void_p, C.c_int]),
    "pt_get_schedule":    (C.c_int, [C.c_void_p]),
    "pt_kernel_time": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), c_int_p]),
    "pt_kernel_time_kind": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_double), c_int_p]),
    "pt_math_eval_device": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    # host (include/pt_host.h)
    "pt_bvh_build": (C.c_int, [C.POINTER(Triangle), C.c_int, C.c_int, C.c_int, C.c_int,
                               C.POINTER(C.POINTER(BvhNodeDevice)), c_int_p, C.POINTER(c_int_p), c_int_p]),
    "pt_bvh_free": (None, [C.POINTER(BvhNodeDevice), c_int_p]),
    "pt_morton_code": (C.c_uint, [C.c_float, C.c_float, C.c_float]),
    "pt_clz_table": (C.c_uint, [C.c_uint]),
    "pt_scene_builder_create": (C.c_void_p, []),
    "pt_scene_builder_destroy": (None, [C.c_void_p]),
    "pt_scene_builder_add_material": (C.c_int, [C.c_void_p, C.POINTER(Material)]),
    "pt_scene_builder_add_sphere": (C.c_int, [C.c_void_p, Float3, C.c_float, C.POINTER(Material)]),
    "pt_scene_builder_add_mesh": (C.c_int, [C.c_void_p, C.c_int, c_float_p, c_float_p, c_float_p, c_int_p, Float3,
                                            Float3, Float3]),
    "pt_scene_builder_set_cube_map": (C.c_int, [C.c_void_p, C.c_int, c_ubyte_p]),
    "pt_scene_builder_add_texture": (C.c_int, [C.c_void_p, C.c_int, C.c_int, c_ubyte_p]),
    "pt_scene_builder_build": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "pt_scene_builder_view": (C.c_int, [C.c_void_p, C.POINTER(SceneView)]),
    "pt_scene_builder_set_transform": (C.c_int, [C.c_void_p, C.c_int, Float3, Float3]),
    "pt_scene_builder_set_rotate": (C.c_int, [C.c_void_p, C.c_int, Float3]),
    "pt_scene_builder_apply_rotate": (C.c_int, [C.c_void_p, C.c_int]),
    "pt_scene_builder_mesh_local": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.POINTER(Triangle)), c_int_p, c_int_p,
                                              C.POINTER(C.POINTER(BoundingBox)), c_int_p, C.POINTER(Float3),
                                              C.POINTER(Float3)]),
    "pt_view_camera_default": (None, [C.POINTER(ViewCamera)]),
    "pt_view_camera_set_resolution": (None, [C.POINTER(ViewCamera), C.c_float, C.c_float]),
    "pt_view_camera_set_fov": (None, [C.POINTER(ViewCamera), C.c_float]),
    "pt_view_camera_get_render_camera": (None, [C.POINTER(ViewCamera), C.POINTER(RenderCamera)]),
    "pt_configuration_default": (None, [C.POINTER(Configuration)]),
    "pt_bvh_build_ex": (C.c_int, [C.POINTER(Triangle), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.POINTER(C.POINTER(BvhNodeDevice)), c_int_p, C.POINTER(c_int_p), c_int_p]),
    "pt_bvh_build_naive": (C.c_int, [C.POINTER(Triangle), C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.POINTER(C.POINTER(BvhNodeDevice)), c_int_p, C.POINTER(c_int_p), c_int_p]),
    "pt_bvh_build_sah": (C.c_int, [C.POINTER(Triangle), C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.POINTER(C.POINTER(BvhNodeDevice)), c_int_p, C.POINTER(c_int_p), c_int_p]),
    "pt_bvh_build_sah_device": (C.c_int, [C.POINTER(Triangle), C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.POINTER(C.POINTER(BvhNodeDevice)), c_int_p, C.POINTER(c_int_p), c_int_p]),
    "pt_scene_builder_build_ex": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int]),
    "pt_scene_builder_set_bvh_device": (C.c_int, [C.c_void_p, C.c_int]),
    # GPU BVH builder (include/pt_bvh.h)
    "compute_triangle_bounding_box_kernel": (None, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    "generate_internal_node_kernel": (None, [C.c_void_p, C.c_uint, C.c_void_p, C.c_uint, C.c_int]),
    "radix_sort": (None, [C.c_void_p, C.c_void_p, C.c_int]),
    "pt_bvh_build_device": (C.c_int, [C.POINTER(Triangle), C.c_int, C.c_int, C.c_int,
                                      C.POINTER(C.POINTER(BvhNodeDevice)), c_int_p, C.POINTER(c_int_p), c_int_p]),
    # ingestion (include/pt_loader.h)
    "pt_config_load": (C.c_int, [C.c_char_p, C.POINTER(Configuration)]),
    "pt_material_preset": (C.c_int, [C.c_char_p, C.POINTER(Material)]),
    "pt_obj_load": (C.c_int, [C.c_char_p, C.POINTER(ObjMesh)]),
    "pt_obj_free": (None, [C.POINTER(ObjMesh)]),
    "pt_scene_load": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(SceneLoadOptions)]),
    "pt_image_load": (C.c_int, [C.c_char_p, c_int_p, c_int_p, C.POINTER(c_ubyte_p)]),
    "pt_image_free": (None, [c_ubyte_p]),
    "pt_jpeg_decode": (C.c_int, [c_ubyte_p, C.c_size_t, C.c_int, c_int_p, c_int_p, C.POINTER(c_ubyte_p)]),
    "pt_image_write_png": (C.c_int, [C.c_char_p, C.c_int, C.c_int, c_ubyte_p, C.c_int]),
}

EXPORTED = tuple(_PROTOS)

_lib = None


def lib() -> C.CDLL:
    """Load libpt_hip.so (building it first if it is absent and hipcc is available)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        from .build import build
        build()
    handle = C.CDLL(LIB, mode=C.RTLD_GLOBAL)
    # PT_ABI_OLD_LIB=1: an earlier round's library loaded for an A/B (PT_LIBDIR); exports it predates are skipped
    lenient = os.environ.get("PT_ABI_OLD_LIB") == "1"
    for name, (res, args) in _PROTOS.items():
        if lenient and not hasattr(handle, name):
            continue
        fn = getattr(handle, name)  # AttributeError = missing export: fail loudly
        fn.restype = res
        fn.argtypes = args
    _lib = handle
    return _lib


class PtError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().pt_last_error()
        raise PtError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
