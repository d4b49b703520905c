"""GPU BVH builder (row f1, include/pt_bvh.h) against the host builder and the reference's
intermediate-node semantics.

* pt_bvh_build_device (bvh_morton_code_cuda::build_bvh, Bvh/bvh.cpp:862-1047) must produce the
  host builder's node array bit for bit (boxes, leaf flags, skip indices, leaf triangle slots):
  equal-code runs, zero-extent meshes, leaf sizes 1-4, large meshes.
* The reference ABI trio — compute_triangle_bounding_box_kernel, radix_sort,
  generate_internal_node_kernel (Kernel/bvh_morton_code_kernel.cu:298-392,
  Kernel/parallel_function.cu:22-32) — on host buffers, checked against the Python restatement in
  tests/test_bvh.py (Morton codes, stable order, Karras children).
"""
import ctypes as C

import numpy as np
import pytest

import pathtracerwithcuda_amd as pt
from pathtracerwithcuda_amd import _abi
from test_bvh import build_py, clz, make_tris, morton_py, run_builder

pytestmark = pytest.mark.gpu
F = np.float32


def tri_array(tris):
    arr = (_abi.Triangle * len(tris))()
    for i, t in enumerate(tris):
        arr[i].vertex0 = _abi.Float3(*map(float, t[0]))
        arr[i].vertex1 = _abi.Float3(*map(float, t[1]))
        arr[i].vertex2 = _abi.Float3(*map(float, t[2]))
    return arr


def run_device_builder(tris, start, leaf_size):
    n = len(tris)
    arr = tri_array(tris)
    nodes = C.POINTER(_abi.BvhNodeDevice)()
    leaf = _abi.c_int_p()
    nn, ln = C.c_int(), C.c_int()
    rc = pt.lib().pt_bvh_build_device(arr, n, start, leaf_size, C.byref(nodes), C.byref(nn), C.byref(leaf), C.byref(ln))
    assert rc == 0
    res = []
    for i in range(nn.value):
        d = nodes[i]
        slots = [d.triangle_indices[k] for k in range(leaf_size)] if d.is_leaf else None
        res.append((bytes(d.box), bool(d.is_leaf), d.next_node_index, slots))
    pt.lib().pt_bvh_free(nodes, leaf)
    return res


def host_as_bytes(tris, start, leaf_size):
    out = []
    for lb, rt, is_leaf, nxt, slots in run_builder(tris, start, leaf_size):
        box = _abi.BoundingBox(_abi.Float3(*map(float, lb)), _abi.Float3(*map(float, rt)),
                               _abi.Float3(*map(float, (F(0.5) * (rt + lb)).astype(F))))
        out.append((bytes(box), is_leaf, nxt, slots))
    return out


@pytest.mark.parametrize("n,leaf,start,kind", [(1, 1, 0, "rand"), (2, 1, 3, "rand"), (300, 1, 0, "rand"),
                                               (301, 2, 10, "rand"), (1000, 4, 3, "rand"), (257, 3, 0, "rand"),
                                               (200, 1, 0, "flat"), (120, 1, 0, "dup"), (20000, 1, 7, "rand"),
                                               (1000, 1, 0, "dup2"), (4096, 1, 0, "same"), (4095, 2, 0, "same"),
                                               (3000, 1, 0, "dupmix"), (3001, 3, 2, "dupmix")])
def test_device_builder_equals_host_builder(require_gpu, n, leaf, start, kind):
    """Equal Morton codes (dup, dup2, same, dupmix) are where the reference's Karras split can give a
    malformed tree — the ADVICE r02 case: a cycle passes the reference counts, and the device finish
    must then take the host finish instead of climbing forever (pt_bvh.hip fin_flatten)."""
    if kind == "dup":
        tris = np.repeat(make_tris(3, 1), n // 3, axis=0)
    elif kind == "dup2":
        tris = np.repeat(make_tris(2, 5), n // 2, axis=0)
    elif kind == "same":
        tris = np.repeat(make_tris(1, 9), n, axis=0)
    elif kind == "dupmix":  # runs of equal codes between distinct ones
        base = make_tris(n // 10 + 1, 11)
        tris = np.concatenate([np.repeat(base[:n // 20 + 1], 5, axis=0), make_tris(n, 13)])[:n]
    else:
        tris = make_tris(n, n * 7 + leaf, kind == "flat")
    tris[:5, 0, 0] = F(-0.0) if n > 5 else tris[:5, 0, 0]  # signed zeros in the folds
    got = run_device_builder(tris, start, leaf)
    want = host_as_bytes(tris, start, leaf)
    assert len(got) == len(want)
    assert got == want


def py_as_bytes(tris, start, leaf_size):
    out = []
    for lb, rt, is_leaf, nxt, slots in build_py(tris, start, leaf_size):
        box = _abi.BoundingBox(_abi.Float3(*map(float, lb)), _abi.Float3(*map(float, rt)),
                               _abi.Float3(*map(float, (F(0.5) * (rt + lb)).astype(F))))
        out.append((bytes(box), is_leaf, nxt, slots))
    return out


@pytest.mark.parametrize("n,leaf,start,kind", [(2, 1, 0, "rand"), (300, 1, 0, "rand"), (301, 2, 10, "rand"),
                                               (1000, 4, 3, "rand"), (200, 1, 0, "flat"), (6000, 1, 5, "rand"), (40000, 1, 0, "rand"),
                                               (120, 1, 0, "dup")])
def test_device_builder_equals_python_restatement(require_gpu, n, leaf, start, kind):
    """Row f1 with the second half on the device (bottom-up boxes by arrival counters, preorder flatten,
    pt_bvh.hip fin_*): the node array equals tests/test_bvh.py::build_py — the independent Python
    restatement of bvh.cpp:862-1047 + :244-330 — byte for byte (boxes with centroids, leaf flags, skip
    indices, leaf triangle slots). The duplicate-code case may be a malformed tree, for which the host
    finish runs instead; the result must be the same either way."""
    if kind == "dup":
        tris = np.repeat(make_tris(3, 1), n // 3, axis=0)
    else:
        tris = make_tris(n, n * 11 + leaf, kind == "flat")
    got = run_device_builder(tris, start, leaf)
    want = py_as_bytes(tris, start, leaf)
    assert len(got) == len(want)
    assert got == want


def test_device_builder_on_the_benchmark_mesh(require_gpu):
    sh = pt.torus_knot(350, 100)
    tris = sh.vertices.astype(F)
    got = run_device_builder(tris, 22, 1)
    want = host_as_bytes(tris, 22, 1)
    assert got == want


def test_scene_builder_uses_the_device_for_morton_cuda(require_gpu):
    a = pt.cornell_scene(pt.torus_knot(120, 40), cube_length=0)  # default: device builder
    b = pt.Scene()
    pt.lib().pt_scene_builder_set_bvh_device(b._b, -1)  # host builder
    walls = [b.add_material(m) for m in ("wall_white", "wall_green", "wall_red", "wall_white", "wall_white")]
    b.add_mesh(pt.cornell_shapes(), walls, position=(0.0, -0.8, 1.0), scale=(0.1, 0.1, 0.3))
    b.add_mesh([pt.cube_shape()], [b.add_material("light")], position=(0.0, 3.1, 0.0), scale=(0.85, 0.05, 0.85))
    b.add_mesh([pt.torus_knot(120, 40)], [b.add_material("diffuse_white")], position=(0.0, 1.55, -1.5),
               scale=(0.7, 0.7, 0.7))
    b.add_sphere((-0.9, 0.0, -0.9), 0.8, "iron")
    b.add_sphere((1.3, 0.0, -0.4), 0.8, "glass")
    b.build()
    va, vb = a.view, b.view
    for m in range(va.mesh_num):
        assert va.mesh_node_num[m] == vb.mesh_node_num[m]
        for i in range(va.mesh_node_num[m]):
            x, y = va.bvh_nodes[m][i], vb.bvh_nodes[m][i]
            assert bytes(x.box) == bytes(y.box) and x.next_node_index == y.next_node_index and x.is_leaf == y.is_leaf
            if x.is_leaf:
                assert x.triangle_indices[0] == y.triangle_indices[0]


def test_reference_build_abi_on_host_buffers(require_gpu):
    """The reference's own build sequence (bvh.cpp:888-972) through the three exported kernels."""
    lib = pt.lib()
    tris = make_tris(500, 9)
    n, start = len(tris), 4
    arr = tri_array(tris)
    lb = tris.min(axis=(0, 1)).astype(F)
    rt = tris.max(axis=(0, 1)).astype(F)
    mesh = _abi.BoundingBox(_abi.Float3(*map(float, lb)), _abi.Float3(*map(float, rt)),
                            _abi.Float3(*map(float, (F(0.5) * (rt + lb)).astype(F))))
    tn = (_abi.BvhNodeMorton * n)()
    lib.compute_triangle_bounding_box_kernel(C.cast(arr, C.c_void_p), n, C.cast(tn, C.c_void_p), C.cast(C.pointer(mesh), C.c_void_p), start, 32)
    codes = []
    for i in range(n):
        b = tn[i].box
        got_lb = np.array([b.left_bottom.x, b.left_bottom.y, b.left_bottom.z], F)
        assert np.array_equal(got_lb, tris[i].min(axis=0)) and tn[i].triangle_index == i + start
        c = (F(0.5) * (tris[i].max(axis=0) + tris[i].min(axis=0))).astype(F)
        with np.errstate(all="ignore"):
            p = ((c - lb) / (rt - lb)).astype(F)
        assert tn[i].morton_code == morton_py(p)
        codes.append(tn[i].morton_code)
    srt = (_abi.BvhNodeMorton * n)()
    lib.radix_sort(C.cast(tn, C.c_void_p), C.cast(srt, C.c_void_p), n)
    order = np.argsort(np.array(codes, np.uint64), kind="stable")
    assert [srt[i].triangle_index for i in range(n)] == [int(k) + start for k in order]
    # leaves = the sorted triangles (leaf size 1), internal nodes from the sorted codes
    leaves = (_abi.BvhNodeMorton * n)()
    C.memmove(leaves, srt, C.sizeof(srt))
    internal = (_abi.BvhNodeMorton * (n - 1))()
    lib.generate_internal_node_kernel(C.cast(internal, C.c_void_p), n - 1, C.cast(leaves, C.c_void_p), n, 32)
    sc = [leaves[i].morton_code for i in range(n)]
    for i in range(n - 1):
        a, b = karras_range(sc, i)
        split = karras_split(sc, a, b)
        x = internal[i]
        assert (x.left_index, x.right_index) == (split, split + 1)
        assert (x.is_left_leaf, x.is_right_leaf) == (int(split == a), int(split + 1 == b))
    assert all(leaves[i].parent_index >= 0 for i in range(n))


def karras_range(codes, i):
    """find_range (Bvh/bvh.cpp:486-570), unsigned wrap-around included."""
    L, M = len(codes), 0xFFFFFFFF
    if i == 0:
        return 0, L - 1
    prev, cur, nxt = codes[i - 1], codes[i], codes[i + 1]
    if prev == cur == nxt:
        j = i
        while 0 < j < L - 1:
            j += 1
            if j >= L - 1 or codes[j] != codes[j + 1]:
                break
        return i, j
    l, r = clz(cur ^ prev), clz(cur ^ nxt)
    d, dmin = (-1, r) if l > r else (1, l)
    lmax = 2
    t = (i + lmax * d) & M
    while t < L and clz(cur ^ codes[t]) > dmin:
        lmax *= 2
        t = (i + lmax * d) & M
    ll, div = 0, 2
    while lmax // div >= 1:
        tt = lmax // div
        t = (i + (ll + tt) * d) & M
        if t < L and clz(cur ^ codes[t]) > dmin:
            ll += tt
        div *= 2
    return (i, i + ll * d) if d == 1 else (i + ll * d, i)


def karras_split(codes, a, b):
    """find_split (Bvh/bvh.cpp:446-481)."""
    fc, lc = codes[a], codes[b]
    if fc == lc:
        return a
    common = clz(fc ^ lc)
    split, step = a, b - a
    while True:
        step = (step + 1) >> 1
        if split + step < b and clz(fc ^ codes[split + step]) > common:
            split += step
        if step <= 1:
            break
    return split


def _sah_nodes(fn, tris, start, leaf_size, bins=32):
    arr = tri_array(tris)
    nodes = C.POINTER(_abi.BvhNodeDevice)()
    leaf = _abi.c_int_p()
    nn, ln = C.c_int(), C.c_int()
    assert fn(arr, len(tris), start, leaf_size, bins, C.byref(nodes), C.byref(nn), C.byref(leaf), C.byref(ln)) == 0
    res = []
    for i in range(nn.value):
        d = nodes[i]
        slots = [d.triangle_indices[k] for k in range(leaf_size)] if d.is_leaf else None
        res.append((bytes(d.box), bool(d.is_leaf), d.next_node_index, slots))
    pt.lib().pt_bvh_free(nodes, leaf)
    return res


@pytest.mark.parametrize("order", ["0", "1", "2", "3", "4", "5", "6"])
@pytest.mark.parametrize("n,leaf,start,kind,bins", [(1, 1, 0, "rand", 32), (2, 1, 3, "rand", 32), (300, 1, 0, "rand", 32),
                                                    (5000, 1, 7, "rand", 32), (4099, 3, 0, "rand", 16),
                                                    (2000, 1, 0, "flat", 32), (777, 2, 0, "dup", 64)])
def test_sah_device_builder_equals_host(require_gpu, monkeypatch, order, n, leaf, start, kind, bins):
    """pt_bvh_build_sah_device (pt_bvh_sah.hip: a level per launch, a workgroup per node, ordered-int LDS bins,
    ballot-scan stable partitions) gives pt_bvh_build_sah's node array byte for byte: boxes, leaf flags, skip indices,
    leaf slots, for every child order, leaf sizes 1-3, zero-extent meshes and runs of identical triangles."""
    monkeypatch.setenv("PT_SAH_ORDER", order)
    tris = make_tris(n, n + leaf, flat=kind == "flat")
    if kind == "dup":
        tris = np.repeat(make_tris(n // 7 + 1, 3), 7, axis=0)[:n]
    L = pt.lib()
    host = _sah_nodes(L.pt_bvh_build_sah, tris, start, leaf, bins)
    dev = _sah_nodes(L.pt_bvh_build_sah_device, tris, start, leaf, bins)
    assert len(dev) == len(host)
    for i, (g, w) in enumerate(zip(dev, host)):
        assert g == w, (i, g, w)


def test_sah_device_builder_on_a_large_mesh(require_gpu):
    """A 300k-triangle knot (the C4 mesh's shape at 3/8 the size): the device tree equals the host tree (the scene
    builder's path for PT_BVH_SAH when a GPU is present)."""
    import time
    knot = pt.torus_knot(600, 250)
    tris = knot.vertices
    L = pt.lib()
    t0 = time.perf_counter()
    dev = _sah_nodes(L.pt_bvh_build_sah_device, tris, 0, 1)
    t_dev = time.perf_counter() - t0
    t0 = time.perf_counter()
    host = _sah_nodes(L.pt_bvh_build_sah, tris, 0, 1)
    t_host = time.perf_counter() - t0
    assert dev == host
    print(f"300k SAH tree: device {t_dev * 1e3:.0f} ms, host {t_host * 1e3:.0f} ms")
