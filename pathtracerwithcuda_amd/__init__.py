"""MI355X-native path tracer: the per-pass radiance loop of BlauHimmel/PathTracerWithCuda
(gpu_path_tracer/Kernel/path_tracer_kernel.cu) as hand-written HIP kernels for gfx950, behind the
reference's own C-ABI (include/path_tracer_kernel.h). See DESIGN.md.
"""
from ._abi import LAYOUT, EXPORTED, PtError, lib  # noqa: F401
from .renderer import Renderer, camera, configuration, device_count  # noqa: F401
from .scene import PRESETS, Scene, Shape, cornell_scene, cornell_spheres_scene, cube_shape, cornell_shapes  # noqa: F401
from .scene import material, torus_knot  # noqa: F401
from .scene import procedural_cube_map  # noqa: F401
from .tiling import FrameGroup, StageWatch, TiledFrame, owned_pixels, owned_rows  # noqa: F401
from .loader import load_config, load_image, load_obj, load_scene, material_preset  # noqa: F401

__all__ = ["Renderer", "Scene", "Shape", "camera", "configuration", "cornell_scene", "torus_knot", "material",
           "PRESETS", "lib", "device_count", "PtError", "TiledFrame", "FrameGroup", "StageWatch", "owned_pixels",
           "owned_rows"]
