"""Scene assembly in the reference's data model: material presets, the Cornell-box assets, procedural
stand-ins for the missing meshes, cube maps, and a thin wrapper over the C++ scene builder
(include/pt_host.h).

Reference: Core/material.cpp:12-577 (presets, registered by name in Core/scene_parser.cpp:675-708),
res/obj/cornell.obj + res/obj/cube.obj (geometry restated below), res/scene/cornell_box_simple.json
(placement). The Stanford bunny / dragon / yokohama skybox are not in the reference checkout
(.MISSING_LARGE_BLOBS), so the benchmark scenes use the procedural mesh and cube map here.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import numpy as np

from . import _abi
from ._abi import Float3, Material, check, lib

# name: (diffuse, emission, specular, transparent, roughness, n, k, absorption, reduced_scattering)
_Z = (0.0, 0.0, 0.0)
PRESETS = {
    # Core/material.cpp:12-241 (metals)
    "titanium": (_Z, _Z, (0.542, 0.497, 0.499), False, 0.3, 2.2670, 3.0385, _Z, _Z),
    "chromium": (_Z, _Z, (0.549, 0.556, 0.554), False, 0.3, 2.3230, 3.1350, _Z, _Z),
    "iron": (_Z, _Z, (0.562, 0.556, 0.578), False, 0.3, 2.5845, 2.7670, _Z, _Z),
    "nickel": (_Z, _Z, (0.662, 0.609, 0.526), False, 0.3, 1.7290, 2.9435, _Z, _Z),
    "platinum": (_Z, _Z, (0.673, 0.637, 0.585), False, 0.3, 1.3400, 1.0300, _Z, _Z),
    "copper": (_Z, _Z, (0.955, 0.638, 0.538), False, 0.3, 1.2404, 2.3929, _Z, _Z),
    "palladium": (_Z, _Z, (0.733, 0.697, 0.652), False, 0.3, 1.4080, 3.2540, _Z, _Z),
    "zinc": (_Z, _Z, (0.664, 0.824, 0.850), False, 0.3, 0.67767, 4.01220, _Z, _Z),
    "gold": (_Z, _Z, (1.022, 0.782, 0.344), False, 0.3, 0.89863, 2.4584, _Z, _Z),
    "aluminum": (_Z, _Z, (0.913, 0.922, 0.924), False, 0.3, 0.63324, 5.4544, _Z, _Z),
    "silver": (_Z, _Z, (0.972, 0.960, 0.915), False, 0.3, 0.04, 2.6484, _Z, _Z),
    # Core/material.cpp:243-577 (dielectrics)
    "glass": ((1.0, 1.0, 1.0), _Z, (0.045, 0.045, 0.045), True, 0.1, 1.5319, 0.0, _Z, _Z),
    "green_glass": ((1.0, 1.0, 1.0), _Z, (0.045, 0.045, 0.045), True, 0.1, 1.5319, 0.0, (0.8, 0.01, 0.8), _Z),
    "diamond": ((1.0, 1.0, 1.0), _Z, (1.0, 1.0, 1.0), True, 0.01, 2.4392, 0.0, _Z, _Z),
    "red": ((0.87, 0.15, 0.15), _Z, (1.0, 1.0, 1.0), False, 0.01, 1.491, 0.0, _Z, _Z),
    "green": ((0.15, 0.87, 0.15), _Z, (1.0, 1.0, 1.0), False, 0.01, 1.491, 0.0, _Z, _Z),
    "orange": ((0.93, 0.33, 0.04), _Z, (1.0, 1.0, 1.0), False, 0.01, 1.491, 0.0, _Z, _Z),
    "purple": ((0.5, 0.1, 0.9), _Z, (1.0, 1.0, 1.0), False, 0.01, 1.491, 0.0, _Z, _Z),
    "blue": ((0.4, 0.6, 0.8), _Z, (1.0, 1.0, 1.0), False, 0.01, 1.491, 0.0, _Z, _Z),
    "wall_blue": ((0.4, 0.6, 0.8), _Z, _Z, False, 0.01, 1.491, 0.0, _Z, _Z),
    "wall_red": ((0.87, 0.15, 0.15), _Z, _Z, False, 0.01, 1.491, 0.0, _Z, _Z),
    "wall_green": ((0.15, 0.87, 0.15), _Z, _Z, False, 0.01, 1.491, 0.0, _Z, _Z),
    "wall_white": ((1.0, 1.0, 1.0), _Z, _Z, False, 0.01, 1.491, 0.0, _Z, _Z),
    "marble": (_Z, _Z, (1.0, 1.0, 1.0), True, 0.01, 1.486, 0.0, (0.6, 0.6, 0.6), (8.0, 8.0, 8.0)),
    "something_blue": (_Z, _Z, (1.0, 1.0, 1.0), True, 0.01, 1.333, 0.0, (0.9, 0.3, 0.02), (2.0, 2.0, 2.0)),
    "something_red": (_Z, _Z, (1.0, 1.0, 1.0), True, 0.01, 1.35, 0.0, (0.02, 5.1, 5.7), (9.0, 9.0, 9.0)),
    "light": (_Z, (13.0, 13.0, 11.0), _Z, False, 0.01, 1.000293, 0.0, _Z, _Z),
    # scene-JSON materials used by the benchmark configs
    # res/scene/dragon_on_table_jade.json:10-22
    "DragonGreen": (_Z, _Z, (1.0, 1.0, 1.0), True, 0.01, 1.33, 0.0, (40.0, 3.0, 14.0), (400.0, 400.0, 400.0)),
    # "diffuse only" surface for config 2: index-matched to air, so the Fresnel branch never reflects
    "diffuse_white": ((0.8, 0.8, 0.8), _Z, _Z, False, 0.0, 1.000293, 0.0, _Z, _Z),
}
# res/scene/micro_surface.json: silver-like GGX spheres of increasing roughness
for _i, _r in enumerate((0.01, 0.2, 0.4, 0.6, 0.8, 1.0), start=1):
    PRESETS[f"Micro{_i}"] = (_Z, _Z, (0.972, 0.960, 0.915), False, _r, 0.04, 2.6484, _Z, _Z)


def f3(v) -> Float3:
    return Float3(float(v[0]), float(v[1]), float(v[2]))


def material(spec, diffuse_texture_id: int = -1, specular_texture_id: int = -1) -> Material:
    """A reference `material` from a preset name or a 9-tuple as in PRESETS."""
    p = PRESETS[spec] if isinstance(spec, str) else spec
    d, e, s, tr, rough, n, k, ab, rs = p
    m = Material()
    m.diffuse_color, m.emission_color, m.specular_color = f3(d), f3(e), f3(s)
    m.is_transparent = 1 if tr else 0
    m.roughness = float(rough)
    m.medium.refraction_index = float(n)
    m.medium.extinction_coefficient = float(k)
    m.medium.scattering.absorption_coefficient = f3(ab)
    m.medium.scattering.reduced_scattering_coefficient = f3(rs)
    m.diffuse_texture_id = diffuse_texture_id
    m.specular_texture_id = specular_texture_id
    return m


@dataclass
class Shape:
    """One OBJ shape: per-triangle corners (T,3,3), normals (T,3,3), uvs (T,3,2) or None."""
    vertices: np.ndarray
    normals: np.ndarray
    uvs: np.ndarray | None = None


def _quad(corners, normal) -> Shape:
    # cornell.obj faces "a b c" and "c d a" of each wall quad
    a, b, c, d = (np.asarray(p, np.float32) for p in corners)
    v = np.stack([np.stack([a, b, c]), np.stack([c, d, a])]).astype(np.float32)
    n = np.broadcast_to(np.asarray(normal, np.float32), v.shape).copy()
    return Shape(v, n)


def cornell_shapes() -> list[Shape]:
    """res/obj/cornell.obj: BackWall, RightWall, LeftWall, Ceiling, Floor (5 shapes, 10 triangles)."""
    return [
        _quad([(-28, 0, -20), (28, 0, -20), (28, 40, -20), (-28, 40, -20)], (0, 0, 1)),
        _quad([(-28, 0, 20), (-28, 0, -20), (-28, 40, -20), (-28, 40, 20)], (1, 0, 0)),
        _quad([(28, 0, -20), (28, 0, 20), (28, 40, 20), (28, 40, -20)], (-1, 0, 0)),
        _quad([(28, 40, 20), (-28, 40, 20), (-28, 40, -20), (28, 40, -20)], (0, -1, 0)),
        _quad([(28, 0, 20), (28, 0, -20), (-28, 0, -20), (-28, 0, 20)], (0, 1, 0)),
    ]


def cube_shape() -> Shape:
    """res/obj/cube.obj: one shape (pCube1), 12 triangles, +-0.8 box with per-face normals and uvs."""
    P = np.array([(-.8, -.8, .8), (.8, -.8, .8), (-.8, .8, .8), (.8, .8, .8), (-.8, .8, -.8), (.8, .8, -.8),
                  (-.8, -.8, -.8), (.8, -.8, -.8)], np.float32)
    T = np.array([(.375, 0), (.625, 0), (.375, .25), (.625, .25), (.375, .5), (.625, .5), (.375, .75), (.625, .75),
                  (.375, 1), (.625, 1), (.875, 0), (.875, .25), (.125, 0), (.125, .25)], np.float32)
    N = np.array([(0, 0, 1)] * 4 + [(0, 1, 0)] * 4 + [(0, 0, -1)] * 4 + [(0, -1, 0)] * 4 + [(1, 0, 0)] * 4
                 + [(-1, 0, 0)] * 4, np.float32)
    faces = [((1, 1, 1), (2, 2, 2), (3, 3, 3)), ((3, 3, 3), (2, 2, 2), (4, 4, 4)),
             ((3, 3, 5), (4, 4, 6), (5, 5, 7)), ((5, 5, 7), (4, 4, 6), (6, 6, 8)),
             ((5, 5, 9), (6, 6, 10), (7, 7, 11)), ((7, 7, 11), (6, 6, 10), (8, 8, 12)),
             ((7, 7, 13), (8, 8, 14), (1, 9, 15)), ((1, 9, 15), (8, 8, 14), (2, 10, 16)),
             ((2, 2, 17), (8, 11, 18), (4, 4, 19)), ((4, 4, 19), (8, 11, 18), (6, 12, 20)),
             ((7, 13, 21), (1, 1, 22), (5, 14, 23)), ((5, 14, 23), (1, 1, 22), (3, 3, 24))]
    v = np.array([[P[a - 1] for a, _, _ in f] for f in faces], np.float32)
    uv = np.array([[T[b - 1] for _, b, _ in f] for f in faces], np.float32)
    n = np.array([[N[c - 1] for _, _, c in f] for f in faces], np.float32)
    return Shape(v, n, uv)


def torus_knot(tubular: int = 350, radial: int = 100, p: int = 2, q: int = 3, radius: float = 1.0,
               tube: float = 0.3, uv_repeat: float = 0.0) -> Shape:
    """Procedural (p,q) torus knot with 2*tubular*radial triangles and analytic tube normals.

    Stands in for the ~70k-triangle Stanford bunny of config 2 (350x100x2 = 70,000) and, at
    1000x400x2 = 800,000, for the dragon of config 4 (both absent from the reference checkout).
    """
    u = np.arange(tubular, dtype=np.float64) / tubular * p * 2 * math.pi
    v = np.arange(radial, dtype=np.float64) / radial * 2 * math.pi

    def curve(t):
        cu, su, qr = np.cos(t), np.sin(t), q / p * t
        r = radius * (2 + np.cos(qr)) * 0.5
        return np.stack([r * cu, r * su, radius * np.sin(qr) * 0.5], -1)

    p1 = curve(u)
    p2 = curve(u + 0.01)
    T = p2 - p1
    Nn = p2 + p1
    B = np.cross(T, Nn)
    Nn = np.cross(B, T)
    B /= np.linalg.norm(B, axis=-1, keepdims=True)
    Nn /= np.linalg.norm(Nn, axis=-1, keepdims=True)
    cx = -tube * np.cos(v)[None, :, None]
    cy = tube * np.sin(v)[None, :, None]
    off = cx * Nn[:, None, :] + cy * B[:, None, :]
    pos = p1[:, None, :] + off                           # (tubular, radial, 3)
    nrm = off / np.linalg.norm(off, axis=-1, keepdims=True)
    i = np.arange(tubular)[:, None]
    j = np.arange(radial)[None, :]
    i1 = (i + 1) % tubular
    j1 = (j + 1) % radial
    a = (i, j); b = (i1, j); c = (i1, j1); d = (i, j1)
    idx = [(a, b, d), (b, c, d)]
    V = np.concatenate([np.stack([pos[x] for x in tri], axis=2).reshape(-1, 3, 3) for tri in idx])
    Nr = np.concatenate([np.stack([nrm[x] for x in tri], axis=2).reshape(-1, 3, 3) for tri in idx])
    uvs = None
    if uv_repeat > 0:  # texture coordinates along (u: the knot, v: around the tube), `uv_repeat` tiles per loop
        tu = np.broadcast_to((np.arange(tubular + 1)[:, None] / tubular * uv_repeat), (tubular + 1, radial + 1))
        tv = np.broadcast_to((np.arange(radial + 1)[None, :] / radial), (tubular + 1, radial + 1))
        tex = np.stack([tu, tv], -1)
        ii, jj = np.arange(tubular)[:, None], np.arange(radial)[None, :]
        ta, tb, tc, td = (ii, jj), (ii + 1, jj), (ii + 1, jj + 1), (ii, jj + 1)  # unwrapped (no modulo)
        uvs = np.concatenate([np.stack([tex[x] for x in tri], axis=2).reshape(-1, 3, 2)
                              for tri in [(ta, tb, td), (tb, tc, td)]]).astype(np.float32)
    return Shape(V.astype(np.float32), Nr.astype(np.float32), uvs)


def procedural_cube_map(length: int = 512, seed: int = 7) -> np.ndarray:
    """Six RGBA8 faces (x+, x-, y+, y-, z+, z-), top row first: a sky gradient with a tiled pattern.

    Stands in for the missing `yokohama` skybox (cornell_box_simple.json:3-7) at the size of the
    present 512^2 BMP skyboxes (lobby/lake/hexagon)."""
    rng = np.random.default_rng(seed)
    faces = np.empty((6, length, length, 4), np.uint8)
    yy, xx = np.meshgrid(np.linspace(0, 1, length), np.linspace(0, 1, length), indexing="ij")
    for f in range(6):
        base = rng.uniform(0.25, 0.9, 3)
        check_ = ((np.floor(xx * 8) + np.floor(yy * 8)) % 2) * 0.15
        for ch in range(3):
            val = base[ch] * (0.55 + 0.45 * (1 - yy)) + check_
            faces[f, :, :, ch] = np.clip(val * 255, 0, 255).astype(np.uint8)
        faces[f, :, :, 3] = 255
    return faces


class Scene:
    """Reference-layout scene owned by the C++ builder (pt_scene_builder_*)."""

    def __init__(self):
        self._lib = lib()
        self._b = self._lib.pt_scene_builder_create()
        self._view = None
        self.material_names: list[str] = []
        self.triangle_count = 0

    def close(self):
        if self._b:
            self._lib.pt_scene_builder_destroy(self._b)
            self._b = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_material(self, spec, name: str | None = None, **tex) -> int:
        m = spec if isinstance(spec, Material) else material(spec, **tex)
        mid = self._lib.pt_scene_builder_add_material(self._b, C.byref(m))
        if mid < 0:
            raise _abi.PtError("add_material failed")
        self.material_names.append(name or (spec if isinstance(spec, str) else f"m{mid}"))
        self._view = None
        return mid

    def add_sphere(self, center, radius: float, spec) -> int:
        m = spec if isinstance(spec, Material) else material(spec)
        sid = self._lib.pt_scene_builder_add_sphere(self._b, f3(center), float(radius), C.byref(m))
        self._view = None
        return sid

    def add_mesh(self, shapes: list[Shape], materials: list[int], position=(0, 0, 0), scale=(1, 1, 1),
                 rotate=(0, 0, 0)) -> int:
        """shapes[i] gets materials[min(i, len-1)] (triangle_mesh.cpp:54-185)."""
        if not materials:
            raise ValueError("a mesh needs at least one material (triangle_mesh.cpp:10-14)")
        V = np.ascontiguousarray(np.concatenate([s.vertices for s in shapes]).reshape(-1), np.float32)
        N = np.ascontiguousarray(np.concatenate([s.normals for s in shapes]).reshape(-1), np.float32)
        has_uv = all(s.uvs is not None for s in shapes)
        UV = np.ascontiguousarray(np.concatenate([s.uvs for s in shapes]).reshape(-1), np.float32) if has_uv else None
        mats = np.concatenate([np.full(len(s.vertices), materials[min(i, len(materials) - 1)], np.int32)
                               for i, s in enumerate(shapes)])
        n = len(mats)
        mid = self._lib.pt_scene_builder_add_mesh(
            self._b, n, V.ctypes.data_as(_abi.c_float_p), N.ctypes.data_as(_abi.c_float_p),
            UV.ctypes.data_as(_abi.c_float_p) if UV is not None else None, mats.ctypes.data_as(_abi.c_int_p),
            f3(position), f3(scale), f3(rotate))
        if mid < 0:
            raise _abi.PtError("add_mesh failed")
        self.triangle_count += n
        self._view = None
        return mid

    def set_cube_map(self, faces: np.ndarray) -> None:
        faces = np.ascontiguousarray(faces, np.uint8)
        assert faces.ndim == 4 and faces.shape[0] == 6 and faces.shape[1] == faces.shape[2] and faces.shape[3] == 4
        check(self._lib.pt_scene_builder_set_cube_map(self._b, faces.shape[1], faces.ctypes.data_as(_abi.c_ubyte_p)),
              "set_cube_map")
        self._view = None

    def add_texture(self, rgba: np.ndarray) -> int:
        rgba = np.ascontiguousarray(rgba, np.uint8)
        tid = self._lib.pt_scene_builder_add_texture(self._b, rgba.shape[1], rgba.shape[0],
                                                     rgba.ctypes.data_as(_abi.c_ubyte_p))
        self._view = None
        return tid

    def build(self, leaf_size: int = 1, method: int = 2) -> "Scene":
        check(self._lib.pt_scene_builder_build(self._b, leaf_size, method), "scene build")
        v = _abi.SceneView()
        check(self._lib.pt_scene_builder_view(self._b, C.byref(v)), "scene view")
        self._view = v
        return self

    @property
    def view(self) -> _abi.SceneView:
        if self._view is None:
            raise _abi.PtError("scene not built")
        return self._view

    # ---- interactive edits (Core/triangle_mesh.cpp:271-426, Bvh/bvh.cpp:332-356) ----
    def set_transform(self, mesh: int, position, scale) -> None:
        """triangle_mesh::set_transform_device + update_bvh: re-transform the mesh and refit its boxes."""
        check(self._lib.pt_scene_builder_set_transform(self._b, mesh, f3(position), f3(scale)), "set_transform")

    def set_rotate(self, mesh: int, rotate) -> None:
        check(self._lib.pt_scene_builder_set_rotate(self._b, mesh, f3(rotate)), "set_rotate")

    def apply_rotate(self, mesh: int) -> None:
        """triangle_mesh::apply_rotate: rotate the mesh-local triangles and rebuild the mesh's BVH."""
        check(self._lib.pt_scene_builder_apply_rotate(self._b, mesh), "apply_rotate")
        v = _abi.SceneView()
        check(self._lib.pt_scene_builder_view(self._b, C.byref(v)), "scene view")  # node arrays moved
        self._view = v

    def mesh_local(self, mesh: int) -> dict:
        """Mesh-local triangles, initial boxes and their transform (what Renderer.attach_mesh uploads)."""
        tris, boxes = C.POINTER(_abi.Triangle)(), C.POINTER(_abi.BoundingBox)()
        start, count, nodes = C.c_int(), C.c_int(), C.c_int()
        pos, scl = _abi.Float3(), _abi.Float3()
        check(self._lib.pt_scene_builder_mesh_local(self._b, mesh, C.byref(tris), C.byref(start), C.byref(count),
                                                    C.byref(boxes), C.byref(nodes), C.byref(pos), C.byref(scl)),
              "mesh_local")
        return {"triangles": tris, "tri_start": start.value, "tri_count": count.value, "init_boxes": boxes,
                "node_count": nodes.value, "init_position": pos, "init_scale": scl}

    def node_count(self) -> int:
        v = self.view
        return sum(v.mesh_node_num[i] for i in range(v.mesh_num))


def cornell_spheres_scene(cube_length: int = 512) -> Scene:
    """Config 1: a spheres-only Cornell box (five r=1000 wall spheres, a light sphere, iron + glass
    spheres of cornell_box_simple.json). No BVH. The camera must be inside the box: use
    camera(..., radius=11.0, pitch=0.05, center=(0, 1.2, 0))."""
    s = Scene()
    R = 1000.0
    s.add_sphere((0.0, -0.8 - R, 0.0), R, "wall_white")    # floor
    s.add_sphere((0.0, 3.2 + R, 0.0), R, "wall_white")     # ceiling
    s.add_sphere((0.0, 0.0, -5.0 - R), R, "wall_white")    # back
    s.add_sphere((-2.8 - R, 0.0, 0.0), R, "wall_green")    # left
    s.add_sphere((2.8 + R, 0.0, 0.0), R, "wall_red")       # right
    s.add_sphere((0.0, 3.2 + 0.6, 0.0), 0.75, "light")     # light cap poking through the ceiling
    s.add_sphere((-0.9, 0.0, -0.9), 0.8, "iron")
    s.add_sphere((1.3, 0.0, -0.4), 0.8, "glass")
    if cube_length:
        s.set_cube_map(procedural_cube_map(cube_length))
    return s.build()


def cornell_scene(mesh: Shape | None = None, mesh_material="diffuse_white", mesh_position=(0.0, 1.55, -1.5),
                  mesh_scale=(0.7, 0.7, 0.7), mesh_rotate=(0.0, 0.0, 0.0), spheres: bool = True,
                  cube_length: int = 512, leaf_size: int = 1, method: int = 2) -> Scene:
    """res/scene/cornell_box_simple.json (walls, light, iron + glass spheres) plus an optional mesh. `method`: the BVH
    builder (pt_bvh_build_method: 2 the reference's MortonCodeCUDA, 3 PT_BVH_SAH)."""
    s = Scene()
    walls = [s.add_material(m) for m in ("wall_white", "wall_green", "wall_red", "wall_white", "wall_white")]
    s.add_mesh(cornell_shapes(), walls, position=(0.0, -0.8, 1.0), scale=(0.1, 0.1, 0.3))
    s.add_mesh([cube_shape()], [s.add_material("light")], position=(0.0, 3.1, 0.0), scale=(0.85, 0.05, 0.85))
    if mesh is not None:
        s.add_mesh([mesh], [s.add_material(mesh_material)], position=mesh_position, scale=mesh_scale,
                   rotate=mesh_rotate)
    if spheres:
        s.add_sphere((-0.9, 0.0, -0.9), 0.8, "iron")
        s.add_sphere((1.3, 0.0, -0.4), 0.8, "glass")
    if cube_length:
        s.set_cube_map(procedural_cube_map(cube_length))
    return s.build(leaf_size=leaf_size, method=method)
