"""BVH builder checks (host C++ pt_bvh_build vs an independent Python restatement of
bvh_morton_code_cuda::build_bvh + build_bvh_device_data, Bvh/bvh.cpp:244-330,370-570,862-1047),
Morton/clz known answers, and structural invariants of the flattened skip-pointer array that
the traversal (path_tracer_kernel.cu:85-161) relies on."""
import ctypes as C

import numpy as np
import pytest

import pathtracerwithcuda_amd as pt
from pathtracerwithcuda_amd import _abi

F = np.float32


def expand_bits(v):
    v = (v * 0x00010001) & 0xFF0000FF
    v = (v * 0x00000101) & 0x0F00F00F
    v = (v * 0x00000011) & 0xC30C30C3
    v = (v * 0x00000005) & 0x49249249
    return v & 0xFFFFFFFF


def morton_py(p):
    q = []
    for c in p:
        x = np.float32(c) * F(1024.0)
        x = F(0.0) if np.isnan(x) else x
        q.append(int(min(max(x, F(0.0)), F(1023.0))))
    return (expand_bits(q[0]) * 4 + expand_bits(q[1]) * 2 + expand_bits(q[2])) & 0xFFFFFFFF


def clz(v):
    return 32 - int(v).bit_length()


def build_py(tris, start, leaf_size):
    """Python restatement of the reference builder; returns [(lb, rt, is_leaf, next, tri_slots)]."""
    n = len(tris)
    lb_all = np.minimum.reduce(tris.min(axis=1), axis=0)
    rt_all = np.maximum.reduce(tris.max(axis=1), axis=0)
    boxes = [(t.min(axis=0), t.max(axis=0)) for t in tris]

    def code(b):
        c = (F(0.5) * (b[1] + b[0])).astype(F)
        with np.errstate(all="ignore"):
            p = ((c - lb_all) / (rt_all - lb_all)).astype(F)
        return morton_py(p)

    order = sorted(range(n), key=lambda i: code(boxes[i]))  # stable
    # bvh.cpp:866-868, except a mesh smaller than one leaf is one leaf (the reference reads past the
    # sorted array there; pt_bvh_internal.h pt_leaf_count)
    L = 1 if n < leaf_size else max(n // leaf_size, 1) + (0 if n % leaf_size == 0 else 1)
    leaves = []
    for i in range(L):
        s = i * leaf_size
        lb, rt = boxes[order[s]]
        slots = [order[s] + start]
        for j in range(1, leaf_size):
            if s + j < n:
                b = boxes[order[s + j]]
                lb, rt = np.minimum(lb, b[0]), np.maximum(rt, b[1])
                slots.append(order[s + j] + start)
            else:
                slots.append(-1)
        leaves.append([lb, rt, slots, None])
    for lf in leaves:
        lf[3] = code((lf[0], lf[1]))
    leaves.sort(key=lambda lf: lf[3])
    codes = [lf[3] for lf in leaves]
    M = 0xFFFFFFFF

    def find_range(i):
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

    def find_split(a, b):
        fc, lc = codes[a], codes[b]
        if fc == lc:
            return a
        common = clz(fc ^ lc)
        split, step = a, b - a
        while True:
            step = (step + 1) >> 1
            ns = split + step
            if ns < b and clz(fc ^ codes[ns]) > common:
                split = ns
            if step <= 1:
                break
        return split

    inner = [dict(l=None, r=None) for _ in range(L - 1)]
    parent_leaf = [None] * L
    for i in range(L - 1):
        a, b = find_range(i)
        s = find_split(a, b)
        inner[i]["l"] = ("L", s) if s == a else ("I", s)
        inner[i]["r"] = ("L", s + 1) if s + 1 == b else ("I", s + 1)
        for side in ("l", "r"):
            kind, k = inner[i][side]
            if kind == "L":
                parent_leaf[k] = i

    def box(ref):
        kind, k = ref
        if kind == "L":
            return leaves[k][0], leaves[k][1]
        if "box" not in inner[k]:
            bl, br = box(inner[k]["l"]), box(inner[k]["r"])
            inner[k]["box"] = (np.minimum(bl[0], br[0]), np.maximum(bl[1], br[1]))
        return inner[k]["box"]

    root = ("I", 0) if L > 1 else ("L", 0)
    box(root)
    out, stack = [], [root]
    while stack:  # preorder, right pushed first (bvh.cpp:251-281)
        ref = stack.pop()
        kind, k = ref
        if kind == "L":
            lb, rt = leaves[k][0], leaves[k][1]
            if (rt == lb).any() and parent_leaf[k] is not None:
                pb = inner[parent_leaf[k]]["box"]
                lb, rt = np.minimum(lb, pb[0]), np.maximum(rt, pb[1])
            out.append([lb, rt, True, leaves[k][2]])
        else:
            lb, rt = inner[k]["box"]
            out.append([lb, rt, False, None])
            stack.append(inner[k]["r"])
            stack.append(inner[k]["l"])
    # next = first node after the subtree (bvh.cpp:290-303)
    size = [1] * len(out)
    for i in range(len(out) - 1, -1, -1):
        if not out[i][2]:
            j = i + 1
            j2 = j + size[j]
            size[i] = 1 + size[j] + size[j2]
    return [(o[0], o[1], o[2], i + size[i], o[3]) for i, o in enumerate(out)]


def make_tris(n, seed, flat=False):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-2, 2, (n, 1, 3))
    t = (c + rng.uniform(-0.3, 0.3, (n, 3, 3))).astype(F)
    if flat:
        t[:, :, 1] = F(0.5)  # zero mesh extent in y -> NaN Morton coordinate -> 0
    return t


def run_builder(tris, start, leaf_size):
    n = len(tris)
    arr = (_abi.Triangle * n)()
    for i, t in enumerate(tris):
        arr[i].vertex0 = _abi.Float3(*map(float, t[0]))
        arr[i].vertex1 = _abi.Float3(*map(float, t[1]))
        arr[i].vertex2 = _abi.Float3(*map(float, t[2]))
    nodes = C.POINTER(_abi.BvhNodeDevice)()
    leaf = _abi.c_int_p()
    nn, ln = C.c_int(), C.c_int()
    rc = pt.lib().pt_bvh_build(arr, n, start, leaf_size, 2, C.byref(nodes), C.byref(nn), C.byref(leaf), C.byref(ln))
    assert rc == 0
    res = []
    for i in range(nn.value):
        d = nodes[i]
        lb = np.array([d.box.left_bottom.x, d.box.left_bottom.y, d.box.left_bottom.z], F)
        rt = np.array([d.box.right_top.x, d.box.right_top.y, d.box.right_top.z], F)
        slots = [d.triangle_indices[k] for k in range(leaf_size)] if d.is_leaf else None
        res.append((lb, rt, bool(d.is_leaf), d.next_node_index, slots))
    pt.lib().pt_bvh_free(nodes, leaf)
    return res


@pytest.mark.parametrize("n,leaf,start,flat", [(1, 1, 0, False), (2, 1, 0, False), (7, 1, 5, False),
                                               (300, 1, 0, False), (301, 2, 10, False), (257, 3, 0, False),
                                               (200, 1, 0, True), (1000, 4, 3, False)])
def test_builder_matches_python_restatement(n, leaf, start, flat):
    tris = make_tris(n, n * 7 + leaf, flat)
    got = run_builder(tris, start, leaf)
    want = build_py(tris, start, leaf)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert np.array_equal(g[0], w[0]) and np.array_equal(g[1], w[1])
        assert g[2] == w[2] and g[3] == w[3] and g[4] == w[4]


def test_duplicate_morton_codes_terminate():
    # many identical triangles: equal codes exercise find_range's equal-run branch
    t = np.repeat(make_tris(3, 1), 40, axis=0)
    got = run_builder(t, 0, 1)
    assert got[0][3] == len(got)


def test_morton_and_clz_known_answers():
    L = pt.lib()
    assert L.pt_morton_code(0.0, 0.0, 0.0) == 0
    assert L.pt_morton_code(1.0, 1.0, 1.0) == 0x3FFFFFFF
    assert L.pt_morton_code(1.0, 0.0, 0.0) == 0x24924924
    assert L.pt_morton_code(0.0, 0.0, 1.0) == 0x09249249
    assert L.pt_morton_code(float("nan"), 2.0, -1.0) == expand_bits(1023) * 2
    for v in (0, 1, 2, 3, 255, 256, 65535, 65536, 1 << 24, 0xFFFFFFFF):
        assert L.pt_clz_table(v) == clz(v)


@pytest.mark.parametrize("method,leaf,order", [(2, 1, "0"), (3, 1, "0"), (3, 1, "1"), (3, 1, "2"), (3, 3, "2"),
                                               (3, 1, "3"), (3, 1, "4"), (3, 1, "5"), (3, 1, "6"), (3, 2, "6"),
                                               (2, 2, "0")])
def test_flattened_structure_invariants(monkeypatch, method, leaf, order):
    """The reference's Morton LBVH (2) and PT_BVH_SAH (3, every child order): preorder with skip indices, every
    triangle in exactly one leaf slot, leaves' boxes holding their triangles, children nested in their parents."""
    monkeypatch.setenv("PT_SAH_ORDER", order)
    sc = pt.cornell_scene(pt.torus_knot(80, 20), cube_length=0, method=method, leaf_size=leaf)
    v = sc.view
    tri_seen = np.zeros(v.triangle_num, int)
    for m in range(v.mesh_num):
        nodes = v.bvh_nodes[m]
        num = v.mesh_node_num[m]
        assert nodes[0].next_node_index == num
        start, cnt = v.mesh_triangle_start[m], v.mesh_triangle_num[m]
        for i in range(num):
            d = nodes[i]
            assert i < d.next_node_index <= num
            if d.is_leaf:
                assert d.next_node_index == i + 1
                slots = [d.triangle_indices[k] for k in range(leaf)]
                assert slots[0] >= 0 and all(t == -1 for t in slots[slots.index(-1):]) if -1 in slots else True
                for t in slots:
                    if t < 0:
                        continue
                    assert start <= t < start + cnt
                    tri_seen[t] += 1
                    tr = v.triangles[t]
                    for p in (tr.vertex0, tr.vertex1, tr.vertex2):
                        assert d.box.left_bottom.x <= p.x <= d.box.right_top.x
                        assert d.box.left_bottom.y <= p.y <= d.box.right_top.y
                        assert d.box.left_bottom.z <= p.z <= d.box.right_top.z
            else:
                # both children nest inside the parent box: the first is the next record, the second follows the
                # first's subtree
                for c in (nodes[i + 1], nodes[nodes[i + 1].next_node_index]):
                    for a in "xyz":
                        assert getattr(c.box.left_bottom, a) >= getattr(d.box.left_bottom, a)
                        assert getattr(c.box.right_top, a) <= getattr(d.box.right_top, a)
    assert (tri_seen == 1).all()


def test_sah_tree_is_deterministic_and_cheaper():
    """PT_BVH_SAH builds the same node array every time, and its surface-area cost (sum over internal nodes of
    SA(node) / SA(root)) is below the reference Morton tree's on the bench knot."""
    def cost(sc, m):
        v = sc.view
        nodes = v.bvh_nodes[m]

        def sa(d):
            x = d.box.right_top.x - d.box.left_bottom.x
            y = d.box.right_top.y - d.box.left_bottom.y
            z = d.box.right_top.z - d.box.left_bottom.z
            return x * y + y * z + z * x
        root = sa(nodes[0])
        return sum(sa(nodes[i]) for i in range(v.mesh_node_num[m]) if not nodes[i].is_leaf) / root

    def dump(sc, m):
        v = sc.view
        return [(d.box.left_bottom.x, d.box.right_top.z, d.next_node_index, d.is_leaf,
                 d.triangle_indices[0] if d.is_leaf else -1)
                for d in (v.bvh_nodes[m][i] for i in range(v.mesh_node_num[m]))]
    knot = pt.torus_knot(60, 20)
    a = pt.cornell_scene(knot, cube_length=0, method=3)
    b = pt.cornell_scene(knot, cube_length=0, method=3)
    ref = pt.cornell_scene(knot, cube_length=0, method=2)
    assert dump(a, 2) == dump(b, 2)
    assert cost(a, 2) < 0.95 * cost(ref, 2), (cost(a, 2), cost(ref, 2))
