"""Host-side driver of the render call — the headless counterpart of Core/path_tracer.cpp:18-99
(init / render / clear) on top of libpt_hip.so's native C-ABI (include/pt_native.h).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import Configuration, RenderCamera, ViewCamera, check, lib
from .scene import Scene


def configuration(**overrides) -> Configuration:
    """res/configuration/config.json defaults (pt_configuration_default) with field overrides."""
    cfg = Configuration()
    lib().pt_configuration_default(C.byref(cfg))
    for k, v in overrides.items():
        if not hasattr(cfg, k):
            raise AttributeError(f"configuration has no field {k!r}")
        if k in ("air_absorption_coef", "air_reduced_scattering_coef"):
            v = _abi.Float3(*map(float, v))
        setattr(cfg, k, v)
    return cfg


def camera(width: int, height: int, fov: float = 45.0, yaw: float = 0.0, pitch: float = 0.3, radius: float = 14.0,
           center=(0.0, 0.0, 0.0), aperture: float = 0.0, focal: float | None = None) -> RenderCamera:
    """view_camera defaults (Core/camera.cpp:3-14) -> render_camera (:80-98); FOV as window.cpp:356-360."""
    vc = ViewCamera()
    L = lib()
    L.pt_view_camera_default(C.byref(vc))
    vc.center = _abi.Float3(*map(float, center))
    vc.yaw, vc.pitch, vc.radius = float(yaw), float(pitch), float(radius)
    vc.aperture_radius = float(aperture)
    vc.focal_distance = float(radius if focal is None else focal)
    L.pt_view_camera_set_resolution(C.byref(vc), float(width), float(height))
    L.pt_view_camera_set_fov(C.byref(vc), float(fov))
    rc = RenderCamera()
    L.pt_view_camera_get_render_camera(C.byref(vc), C.byref(rc))
    return rc


def _device_ptr(x) -> int | None:
    """A device buffer as an address: an int, or a tensor's data_ptr() (None / 0 stay null)."""
    if x is None:
        return None
    return int(x.data_ptr()) if hasattr(x, "data_ptr") else int(x)


def deal_bands(ranked: list[int], n: int, regions: int) -> list[int]:
    """Band order for `n` local bands (positions n - len(ranked) .. n - 1 beyond the ranked ones keep
    their band: the partial last band) whose units a launch cuts into `regions` equal contiguous
    regions: position p belongs to the region holding its midpoint, and the ranked bands go out
    round-robin over the regions, each filling its positions front to back."""
    slots: list[list[int]] = [[] for _ in range(regions)]
    for p in range(len(ranked)):
        slots[min(regions - 1, (2 * p + 1) * regions // (2 * n))].append(p)
    order = list(range(n))
    fill = [0] * regions
    r = 0
    for b in ranked:
        while fill[r] == len(slots[r]):
            r = (r + 1) % regions
        order[slots[r][fill[r]]] = b
        fill[r] += 1
        r = (r + 1) % regions
    return order


class Renderer:
    """One device context: resident scene, resident accumulation image, one HIP stream."""

    def __init__(self, device: int = 0):
        self._lib = lib()
        ctx = C.c_void_p()
        check(self._lib.pt_context_create(int(device), C.byref(ctx)), "pt_context_create")
        self._ctx = ctx
        self.width = self.height = 0

    def close(self):
        if self._ctx:
            self._lib.pt_context_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, scene: Scene, config: Configuration) -> None:
        v = scene.view
        check(self._lib.pt_scene_upload(self._ctx, v.mesh_num, v.bvh_nodes, v.triangles, v.triangle_num,
                                        v.sphere_num, v.spheres, v.sky_cube_map, v.mesh_textures, v.texture_num,
                                        C.byref(config)), "pt_scene_upload")

    def scene_info(self) -> dict:
        b, n, t = C.c_longlong(), C.c_int(), C.c_int()
        check(self._lib.pt_scene_info(self._ctx, C.byref(b), C.byref(n), C.byref(t)), "pt_scene_info")
        return {"device_bytes": b.value, "nodes": n.value, "triangles": t.value}

    def last_kernel(self) -> str:
        """The pass kernel configuration the last render launched (e.g. pass_kernel_u<MINW=7,...>)."""
        v = self._lib.pt_last_kernel(self._ctx)
        return v.decode() if v else ""

    def set_medium_bound(self, on) -> None:
        """Tolerance mode: in-medium segments walk with min_t starting at their free-flight distance
        (pt_set_medium_bound; None = the PT_MEDIUM_BOUND environment variable, the default: off)."""
        check(self._lib.pt_set_medium_bound(self._ctx, -1 if on is None else int(bool(on))), "pt_set_medium_bound")

    def set_grid_share(self, percent: int) -> None:
        """Percentage of the occupancy-sized grid this context's pass launches take (frames in flight)."""
        check(self._lib.pt_set_grid_share(self._ctx, int(percent)), "pt_set_grid_share")

    def band_count(self) -> tuple[int, bool]:
        """(bands of this context's share under its tiling, whether the last one is partial)."""
        n, p = C.c_int(), C.c_int()
        check(self._lib.pt_band_count(self._ctx, C.byref(n), C.byref(p)), "pt_band_count")
        return n.value, bool(p.value)

    def set_band_order(self, order) -> None:
        """Hand out local band order[i] i-th (None: row order). Results do not depend on it."""
        if order is None:
            check(self._lib.pt_set_band_order(self._ctx, None, 0), "pt_set_band_order")
            return
        a = (C.c_int * len(order))(*[int(x) for x in order])
        check(self._lib.pt_set_band_order(self._ctx, a, len(order)), "pt_set_band_order")

    def measure_band_cost(self, on: bool) -> None:
        """Zero and start (True) or stop (False) the per-band ray-segment counters."""
        check(self._lib.pt_band_cost_enable(self._ctx, int(bool(on))), "pt_band_cost_enable")

    def band_cost(self) -> list[int]:
        """Ray segments per local band since measure_band_cost(True) (waits for the context's work)."""
        n, _ = self.band_count()
        a = (C.c_uint * n)()
        check(self._lib.pt_band_cost(self._ctx, a, n), "pt_band_cost")
        return [int(x) for x in a]

    def order_bands_by_cost(self, cam: RenderCamera, config: Configuration, passes: int,
                            regions: int = 1) -> list[int]:
        """Render one (untimed) frame measuring each band's ray segments, then hand the bands out most
        expensive first (a partial last band stays last). Returns the order.

        regions > 1: the launch cuts its units into that many contiguous regions (PT_SHARDS = 8, one
        per XCD, pt_work.h), each handed out front to back; the ranked bands are then dealt round-robin
        over the regions' band slots, so that every region starts on its most expensive bands."""
        self.set_band_order(None)
        self.measure_band_cost(True)
        self.render(cam, config, 1, passes, write_u8=0)
        cost = self.band_cost()
        self.measure_band_cost(False)
        n, partial = self.band_count()
        full = n - 1 if partial else n
        ranked = sorted(range(full), key=lambda b: (-cost[b], b))
        order = deal_bands(ranked, n, regions) if regions > 1 else ranked + ([n - 1] if partial else [])
        self.set_band_order(order)
        return order

    def attach_mesh(self, scene: Scene, mesh: int) -> None:
        """Keep mesh `mesh`'s local triangles and initial boxes on the device for set_mesh_transform."""
        d = scene.mesh_local(mesh)
        check(self._lib.pt_mesh_attach(self._ctx, mesh, d["triangles"], d["tri_start"], d["tri_count"], d["init_boxes"],
                                       d["node_count"], d["init_position"], d["init_scale"]), "pt_mesh_attach")

    def set_mesh_transform(self, mesh: int, position, scale) -> None:
        """Re-transform an attached mesh and refit its boxes on the device (Bvh/bvh.cpp:332-356)."""
        check(self._lib.pt_mesh_set_transform(self._ctx, mesh, _abi.Float3(*map(float, position)),
                                              _abi.Float3(*map(float, scale))), "pt_mesh_set_transform")

    def setup_frame(self, width: int, height: int, image_device_ptr: int | None = None) -> None:
        check(self._lib.pt_frame_setup(self._ctx, width, height, C.c_void_p(image_device_ptr or 0)), "pt_frame_setup")
        self.width, self.height = width, height

    def set_tiling(self, band_rows: int, band_count: int, band_index: int) -> None:
        check(self._lib.pt_set_tiling(self._ctx, band_rows, band_count, band_index), "pt_set_tiling")

    def render(self, cam: RenderCamera, config: Configuration, first_pass: int = 1, pass_count: int = 1,
               write_u8: int = 2) -> None:
        check(self._lib.pt_render_passes(self._ctx, C.byref(cam), C.byref(config), first_pass, pass_count, write_u8),
              "pt_render_passes")

    def render_frames(self, cams, config: Configuration, images, images256=None, first_pass: int = 1,
                      pass_count: int = 1, write_u8: int = 2) -> None:
        """pt_render_frames: the same passes of len(cams) frames, frame f through cams[f] into the device buffers
        images[f] (width*height float3) and images256[f] (uchar3, optional): one pass launch per batch of
        passes for all of them. Buffers are device pointers (int) or CUDA tensors."""
        n = len(cams)
        if len(images) != n or (images256 is not None and len(images256) != n):
            raise ValueError("one image (and 8-bit image) per camera")
        arr = (RenderCamera * n)(*cams)
        imgs = (C.c_void_p * n)(*[_device_ptr(x) for x in images])
        imgs8 = (C.c_void_p * n)(*[_device_ptr(x) for x in images256]) if images256 is not None else None
        check(self._lib.pt_render_frames(self._ctx, arr, n, C.byref(config), first_pass, pass_count, write_u8, imgs,
                                         imgs8), "pt_render_frames")

    def finalize_u8(self, config: Configuration, passes: int) -> None:
        check(self._lib.pt_finalize_u8(self._ctx, C.byref(config), passes), "pt_finalize_u8")

    def finalize_u8_image(self, config: Configuration, passes: int, image, image256) -> None:
        """8-bit gamma output of a caller's float image (device pointer or CUDA tensor) into image256."""
        check(self._lib.pt_finalize_u8_image(self._ctx, C.byref(config), passes, _device_ptr(image),
                                             _device_ptr(image256)), "pt_finalize_u8_image")

    def synchronize(self) -> None:
        check(self._lib.pt_synchronize(self._ctx), "pt_synchronize")

    def download(self) -> tuple[np.ndarray, np.ndarray]:
        img = np.empty((self.height, self.width, 3), np.float32)
        img8 = np.empty((self.height, self.width, 3), np.uint8)
        check(self._lib.pt_image_download(self._ctx, img.ctypes.data, img8.ctypes.data), "pt_image_download")
        return img, img8

    def stream_handle(self) -> int:
        """The context's HIP stream (for torch.cuda.ExternalStream): work ordered on it follows the passes."""
        return self._lib.pt_stream_handle(self._ctx) or 0

    def image_device_ptr(self) -> int:
        return self._lib.pt_image_device_ptr(self._ctx) or 0

    def stats_reset(self) -> None:
        check(self._lib.pt_stats_reset(self._ctx), "pt_stats_reset")

    def stats(self) -> dict:
        s, n, t = C.c_ulonglong(), C.c_ulonglong(), C.c_ulonglong()
        check(self._lib.pt_stats(self._ctx, C.byref(s), C.byref(n), C.byref(t)), "pt_stats")
        return {"segments": s.value, "nodes": n.value, "tris": t.value}

    def stats_all(self) -> dict:
        a = (C.c_ulonglong * 7)()
        check(self._lib.pt_stats_all(self._ctx, a, 7), "pt_stats_all")
        keys = ("segments", "nodes", "tris", "hit_mesh", "hit_sphere", "miss", "scatter")
        return dict(zip(keys, (int(x) for x in a)))

    def stats_raw(self, n: int = 32) -> list[int]:
        """The context's raw statistics words (stats[16..]: PT_UPROF counters)."""
        a = (C.c_ulonglong * n)()
        check(self._lib.pt_stats_all(self._ctx, a, n), "pt_stats_all")
        return [int(x) for x in a]

    SCHEDULES = {"persistent": 0, "wavefront": 1}

    def set_schedule(self, schedule: str | None) -> None:
        """'persistent' (one launch per pass), 'wavefront' (extend + shade per depth) or None (default)."""
        check(self._lib.pt_set_schedule(self._ctx, -1 if schedule is None else self.SCHEDULES[schedule]),
              "pt_set_schedule")

    def schedule(self) -> str:
        v = self._lib.pt_get_schedule(self._ctx)
        check(min(v, 0), "pt_get_schedule")
        return {0: "persistent", 1: "wavefront"}[v]

    def set_instrumented(self, on: bool) -> None:
        check(self._lib.pt_set_instrumented(self._ctx, 1 if on else 0), "pt_set_instrumented")

    def math_eval_device(self, which: int, x: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        x = np.ascontiguousarray(x, np.float32)
        o0, o1 = np.empty_like(x), np.empty_like(x)
        check(self._lib.pt_math_eval_device(self._ctx, which, x.ctypes.data, len(x), o0.ctypes.data, o1.ctypes.data),
              "pt_math_eval_device")
        return o0, o1

    def kernel_time_kind(self, kind: int) -> tuple[float, int]:
        """kind: 0 single-kernel pass, 1 extend (BVH walk), 2 shade, 3 finalize, -1 all."""
        ms, n = C.c_double(), C.c_int()
        check(self._lib.pt_kernel_time_kind(self._ctx, kind, C.byref(ms), C.byref(n)), "pt_kernel_time_kind")
        return ms.value, n.value

    def kernel_time(self) -> tuple[float, int]:
        ms, n = C.c_double(), C.c_int()
        check(self._lib.pt_kernel_time(self._ctx, C.byref(ms), C.byref(n)), "pt_kernel_time")
        return ms.value, n.value


def device_count() -> int:
    return lib().pt_device_count()
