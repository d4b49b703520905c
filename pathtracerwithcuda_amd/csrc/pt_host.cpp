// pt_host.cpp — host-side C++ around the render call: BVH builder, scene assembly in the
// reference data layout, orbit camera, configuration defaults. See include/pt_host.h.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/pt_host.h"
#include "pt_bvh_common.h"
#include "pt_bvh_internal.h"
#include "../../include/pt_bvh.h"
#include "../../include/pt_native.h"
#include "pt_glm.h"

namespace {

using ptbvh::Box;
using ptbvh::expand;
using ptbvh::is_thin;

inline Box box_of_triangle(const pt_triangle& t) {  // bounding_box::get_bounding_box(v0, v1, v2)
    return ptbvh::box_of_vertices(&t.vertex0.x, &t.vertex1.x, &t.vertex2.x);
}

}  // namespace

extern "C" unsigned int pt_morton_code(float x, float y, float z) { return ptbvh::morton(x, y, z); }
extern "C" unsigned int pt_clz_table(unsigned int value) { return ptbvh::clz32(value); }

// The second half of bvh_morton_code_cuda::build_bvh (Bvh/bvh.cpp:974-1047) and
// bvh_naive_cpu::build_bvh_device_data (:244-330), shared by the host and the device builder
// (pt_bvh_internal.h): bottom-up boxes, then the preorder skip-pointer array.
int pt_morton_finish(PtMortonTree& t, int leaf_size, pt_bvh_node_device** nodes_out, int* node_num_out,
                     int** leaf_out, int* leaf_num_out) {
    const unsigned int leaf_num = t.leaf_num, internal_num = t.internal_num;
    struct BuildNode {
        Box box;
        int left, right, parent;
    };
    std::vector<BuildNode> inner(internal_num);
    for (unsigned int i = 0; i < internal_num; i++) {
        inner[i].left = t.inner_left[i];
        inner[i].right = t.inner_right[i];
        inner[i].parent = t.inner_parent[i];
    }
    std::vector<Box>& leaf_box = t.leaf_box;
    // bottom-up boxes: union of the two children (:817-860), post-order from the root
    auto child_box = [&](int c) -> const Box& { return c <= -2 ? leaf_box[(size_t)(-c - 2)] : inner[(size_t)c].box; };
    if (internal_num > 0) {
        std::vector<std::pair<int, int>> st;
        st.reserve(64);
        st.push_back({0, 0});
        std::vector<char> seen(internal_num, 0);
        while (!st.empty()) {
            auto& top = st.back();
            int id = top.first;
            if (top.second == 0) {
                top.second = 1;
                if (seen[id]) { st.pop_back(); continue; }  // malformed (duplicate-code) trees: visit once
                seen[id] = 1;
                if (inner[id].left >= 0 && !seen[inner[id].left]) st.push_back({inner[id].left, 0});
                if (inner[id].right >= 0 && !seen[inner[id].right]) st.push_back({inner[id].right, 0});
            } else {
                Box b = child_box(inner[id].left);
                expand(b, child_box(inner[id].right));
                inner[id].box = b;
                st.pop_back();
            }
        }
    }

    // flatten: preorder with an explicit stack, right pushed before left (:244-330)
    struct Ref { int id; bool leaf; };
    auto node_box = [&](Ref r) -> Box& { return r.leaf ? leaf_box[(size_t)r.id] : inner[(size_t)r.id].box; };
    auto parent_of = [&](Ref r) -> int { return r.leaf ? t.leaf_parent[(size_t)r.id] : inner[(size_t)r.id].parent; };
    std::vector<Ref> order;
    order.reserve((size_t)leaf_num + internal_num);
    {
        std::vector<Ref> st;
        st.push_back(internal_num > 0 ? Ref{0, false} : Ref{0, true});
        while (!st.empty()) {
            Ref cur = st.back();
            st.pop_back();
            order.push_back(cur);
            if (cur.leaf) {
                int p = parent_of(cur);
                if (p >= 0 && is_thin(node_box(cur))) expand(node_box(cur), inner[(size_t)p].box);
            } else {
                const BuildNode& b = inner[(size_t)cur.id];
                if (b.right != -1) st.push_back(b.right <= -2 ? Ref{-b.right - 2, true} : Ref{b.right, false});
                if (b.left != -1) st.push_back(b.left <= -2 ? Ref{-b.left - 2, true} : Ref{b.left, false});
            }
        }
    }
    // second pass (:283-310): next_node_index = traversal index of the node left on top of the
    // stack after popping node k and before pushing its children (node_num when empty), i.e.
    // the first node after k's subtree.
    const int node_num = (int)order.size();
    std::vector<int> next_index((size_t)node_num, node_num);
    {
        std::vector<int> tidx_inner(internal_num, -1), tidx_leaf(leaf_num, -1);
        for (int k = 0; k < node_num; k++) {
            if (order[(size_t)k].leaf) tidx_leaf[(size_t)order[(size_t)k].id] = k;
            else tidx_inner[(size_t)order[(size_t)k].id] = k;
        }
        std::vector<Ref> st;
        st.push_back(order[0]);
        int k = 0;
        while (!st.empty()) {
            Ref cur = st.back();
            st.pop_back();
            if (!st.empty()) {
                Ref top = st.back();
                next_index[(size_t)k] = top.leaf ? tidx_leaf[(size_t)top.id] : tidx_inner[(size_t)top.id];
            } else {
                next_index[(size_t)k] = node_num;
            }
            if (!cur.leaf) {
                const BuildNode& b = inner[(size_t)cur.id];
                if (b.right != -1) st.push_back(b.right <= -2 ? Ref{-b.right - 2, true} : Ref{b.right, false});
                if (b.left != -1) st.push_back(b.left <= -2 ? Ref{-b.left - 2, true} : Ref{b.left, false});
            }
            k++;
        }
    }

    pt_bvh_node_device* nodes = (pt_bvh_node_device*)std::calloc((size_t)node_num, sizeof(pt_bvh_node_device));
    int leaf_in_order = 0;
    for (int k = 0; k < node_num; k++) if (order[(size_t)k].leaf) leaf_in_order++;
    int* leaf_idx = (int*)std::malloc((size_t)std::max(leaf_in_order, 1) * (size_t)leaf_size * sizeof(int));
    if (!nodes || !leaf_idx) { std::free(nodes); std::free(leaf_idx); return -2; }
    int li = 0;
    for (int k = 0; k < node_num; k++) {
        Ref r = order[(size_t)k];
        const Box& b = node_box(r);
        pt_bvh_node_device& d = nodes[k];
        d.box.left_bottom = {b.lb[0], b.lb[1], b.lb[2]};
        d.box.right_top = {b.rt[0], b.rt[1], b.rt[2]};
        d.box.centroid = {0.5f * (b.rt[0] + b.lb[0]), 0.5f * (b.rt[1] + b.lb[1]), 0.5f * (b.rt[2] + b.lb[2])};
        d.is_leaf = r.leaf ? 1 : 0;
        d.next_node_index = next_index[(size_t)k];
        d.triangle_indices = nullptr;
        if (r.leaf) {
            int batch = t.leaf_batch[(size_t)r.id];
            for (int j = 0; j < leaf_size; j++) leaf_idx[(size_t)li * leaf_size + j] = t.batch_tris[(size_t)batch * leaf_size + j];
            d.triangle_indices = leaf_idx + (size_t)li * leaf_size;
            li++;
        }
    }
    *nodes_out = nodes;
    *node_num_out = node_num;
    *leaf_out = leaf_idx;
    *leaf_num_out = li;
    return 0;
}

// bvh_morton_code_cuda::build_bvh (Bvh/bvh.cpp:862-1047) + bvh_naive_cpu::build_bvh_device_data
// (:244-330), all on the host. thrust::sort with a comparator is a stable merge sort, so std::stable_sort.
extern "C" int pt_bvh_build(const pt_triangle* tris, int n, int start_index, int leaf_size, int method,
                            pt_bvh_node_device** nodes_out, int* node_num_out, int** leaf_out, int* leaf_num_out) {
    (void)method;
    if (!tris || n <= 0 || leaf_size <= 0 || !nodes_out || !node_num_out || !leaf_out || !leaf_num_out) return -1;

    PtMortonTree t;
    t.leaf_num = pt_leaf_count(n, leaf_size);
    t.internal_num = t.leaf_num - 1;

    // mesh box (:889-895)
    Box mesh = box_of_triangle(tris[0]);
    for (int i = 1; i < n; i++) expand(mesh, box_of_triangle(tris[i]));

    // per-triangle box + Morton code (bvh_morton_code_kernel.cu:298-326)
    struct TriNode { Box box; unsigned int code; int tri; };
    std::vector<TriNode> tn((size_t)n);
    for (int i = 0; i < n; i++) {
        tn[i].box = box_of_triangle(tris[i]);
        tn[i].code = ptbvh::morton_of_box(tn[i].box, mesh);
        tn[i].tri = i + start_index;
    }
    std::stable_sort(tn.begin(), tn.end(), [](const TriNode& a, const TriNode& b) { return a.code < b.code; });

    // batch into leaves (:920-955), then sort the leaves by the code of their own box
    struct LeafNode { Box box; unsigned int code; int batch; };
    std::vector<LeafNode> leaves(t.leaf_num);
    t.batch_tris.assign((size_t)t.leaf_num * leaf_size, -1);
    for (unsigned int i = 0; i < t.leaf_num; i++) {
        int s = (int)i * leaf_size;
        leaves[i].box = tn[s].box;
        t.batch_tris[(size_t)i * leaf_size] = tn[s].tri;
        for (int j = 1; j < leaf_size; j++) {
            if (j + s < n) {
                expand(leaves[i].box, tn[j + s].box);
                t.batch_tris[(size_t)i * leaf_size + j] = tn[j + s].tri;
            }
        }
        leaves[i].code = ptbvh::morton_of_box(leaves[i].box, mesh);
        leaves[i].batch = (int)i;
    }
    std::stable_sort(leaves.begin(), leaves.end(), [](const LeafNode& a, const LeafNode& b) { return a.code < b.code; });

    // Karras internal nodes (bvh_morton_code_kernel.cu:262-296), sequential in index order: the
    // last writer of a parent link is the largest internal index
    std::vector<unsigned int> codes(t.leaf_num);
    t.leaf_box.resize(t.leaf_num);
    t.leaf_batch.resize(t.leaf_num);
    for (unsigned int i = 0; i < t.leaf_num; i++) {
        codes[i] = leaves[i].code;
        t.leaf_box[i] = leaves[i].box;
        t.leaf_batch[i] = leaves[i].batch;
    }
    t.inner_left.assign(t.internal_num, -1);
    t.inner_right.assign(t.internal_num, -1);
    t.inner_parent.assign(t.internal_num, -1);
    t.leaf_parent.assign(t.leaf_num, -1);
    for (unsigned int i = 0; i < t.internal_num; i++) {
        unsigned int rx, ry;
        ptbvh::find_range(codes, t.leaf_num, i, &rx, &ry);
        unsigned int split = ptbvh::find_split(codes, rx, ry);
        if (split == rx) { t.inner_left[i] = -((int)split + 2); t.leaf_parent[split] = (int)i; }
        else { t.inner_left[i] = (int)split; t.inner_parent[split] = (int)i; }
        if (split + 1 == ry) { t.inner_right[i] = -((int)(split + 1) + 2); t.leaf_parent[split + 1] = (int)i; }
        else { t.inner_right[i] = (int)(split + 1); t.inner_parent[split + 1] = (int)i; }
    }
    return pt_morton_finish(t, leaf_size, nodes_out, node_num_out, leaf_out, leaf_num_out);
}

extern "C" void pt_bvh_free(pt_bvh_node_device* nodes, int* leaf_indices) {
    std::free(nodes);
    std::free(leaf_indices);
}

// ---- bvh_naive_cpu (Bvh/bvh.cpp:16-330): bucketed "SAH" split, then the same preorder flattening --
namespace {

using GNode = PtTreeNode;

inline float centroid_axis(const Box& b, int axis) { return 0.5f * (b.rt[axis] + b.lb[axis]); }
inline void box_of_box(Box& dst, const Box& src) { dst = src; }
inline float surface_area(const Box& b) {  // bounding_box::get_surface_area: 2 * volume (bounding_box.h:63-66)
    return 2.0f * (b.rt[0] - b.lb[0]) * (b.rt[1] - b.lb[1]) * (b.rt[2] - b.lb[2]);
}
inline Box default_box() {  // bounding_box() (bounding_box.h:15-26)
    Box b;
    for (int k = 0; k < 3; k++) { b.lb[k] = -1.0f; b.rt[k] = -1.0f; }
    return b;
}
// x86 cvttss2si: NaN and out-of-range values become INT_MIN (the reference's static_cast<int> of
// (centroid - lb) / 0 on a zero-length axis)
inline int trunc_to_int(float x) {
    if (!(x >= -2147483648.0f && x < 2147483648.0f)) return (int)0x80000000u;
    return (int)x;
}

void naive_split(std::vector<GNode>& nodes, const std::vector<Box>& boxes, int start, int leaf_size, int buckets_max) {
    std::vector<int> stack{0};
    std::vector<std::vector<int>> bucket_tris[3];
    std::vector<Box> bucket_box[3];
    std::vector<char> init(std::max(buckets_max, 1));
    while (!stack.empty()) {
        const int cur = stack.back();
        stack.pop_back();
        int split_axis = -1, split_i = 0, split_div = 0, nl = 0, nr = 0;
        Box bl{}, br{};
        float min_cost = INFINITY;
        const std::vector<int> tris = nodes[(size_t)cur].tris;
        const Box cbox = nodes[(size_t)cur].box;
        for (int axis = 0; axis < 3; axis++) {
            const float axis_length = cbox.rt[axis] - cbox.lb[axis];
            const int div = std::min(buckets_max, (int)tris.size());
            const float internal_length = axis_length / (float)div;
            bucket_tris[axis].assign((size_t)div, {});
            bucket_box[axis].assign((size_t)div, default_box());
            std::fill(init.begin(), init.end(), 0);
            for (int t : tris) {
                const Box& tb = boxes[(size_t)(t - start)];
                int k = trunc_to_int((centroid_axis(tb, axis) - cbox.lb[axis]) / internal_length);
                k = k >= div ? div - 1 : (k < 0 ? 0 : k);
                if (!init[k]) { box_of_box(bucket_box[axis][k], tb); init[k] = 1; }
                else expand(bucket_box[axis][k], tb);
                bucket_tris[axis][k].push_back(t);
            }
            for (int i = 0; i < div; i++) {
                Box left = default_box(), right = default_box();
                size_t cl = 0, cr = 0;
                for (int j = 0; j < i; j++) if (init[j]) { box_of_box(left, bucket_box[axis][j]); break; }
                for (int j = 0; j < i; j++)
                    if (init[j]) { expand(left, bucket_box[axis][j]); cl += bucket_tris[axis][j].size(); }
                for (int j = i; j < div; j++) if (init[j]) { box_of_box(right, bucket_box[axis][j]); break; }
                for (int j = i; j < div; j++)
                    if (init[j]) { expand(right, bucket_box[axis][j]); cr += bucket_tris[axis][j].size(); }
                const float cost = surface_area(left) * (float)cl + surface_area(right) * (float)cr;
                if (cost < min_cost && cost > 0.0f) {
                    min_cost = cost; split_axis = axis; split_i = i; split_div = div;
                    bl = left; br = right; nl = (int)cl; nr = (int)cr;
                }
            }
        }
        std::vector<int> lt, rt;
        if (split_axis >= 0 && nl > 0 && nr > 0) {
            for (int i = 0; i < split_i; i++)
                lt.insert(lt.end(), bucket_tris[split_axis][i].begin(), bucket_tris[split_axis][i].end());
            for (int i = split_i; i < split_div; i++)
                rt.insert(rt.end(), bucket_tris[split_axis][i].begin(), bucket_tris[split_axis][i].end());
        } else {
            // No split with positive cost (planar geometry: every "surface area" is a zero volume), or a
            // split that leaves one side empty: the reference then reads uninitialised split state or
            // re-splits the same node forever. Defined here: halve the node's triangle list.
            const size_t h = tris.size() / 2;
            lt.assign(tris.begin(), tris.begin() + h);
            rt.assign(tris.begin() + h, tris.end());
            bl = boxes[(size_t)(lt[0] - start)];
            for (int t : lt) expand(bl, boxes[(size_t)(t - start)]);
            br = boxes[(size_t)(rt[0] - start)];
            for (int t : rt) expand(br, boxes[(size_t)(t - start)]);
        }
        for (int side = 0; side < 2; side++) {
            GNode child;
            child.box = side == 0 ? bl : br;
            child.tris = side == 0 ? lt : rt;
            child.parent = cur;
            child.leaf = (int)child.tris.size() <= leaf_size;
            if (child.leaf) child.tris.resize((size_t)leaf_size, -1);
            const int id = (int)nodes.size();
            nodes.push_back(std::move(child));
            (side == 0 ? nodes[(size_t)cur].left : nodes[(size_t)cur].right) = id;
            if (!nodes[(size_t)id].leaf) stack.push_back(id);
        }
    }
}

// build_bvh_device_data (Bvh/bvh.cpp:244-330) over a linked tree rooted at node 0.
int flatten_tree(std::vector<GNode>& nodes, int leaf_size, pt_bvh_node_device** nodes_out, int* node_num_out,
                 int** leaf_out, int* leaf_num_out) {
    std::vector<int> order, tindex(nodes.size(), -1);
    {
        std::vector<int> st{0};
        while (!st.empty()) {
            const int cur = st.back();
            st.pop_back();
            tindex[(size_t)cur] = (int)order.size();
            order.push_back(cur);
            GNode& g = nodes[(size_t)cur];
            if (g.leaf && g.parent >= 0 && is_thin(g.box)) expand(g.box, nodes[(size_t)g.parent].box);
            if (g.right != -1) st.push_back(g.right);
            if (g.left != -1) st.push_back(g.left);
        }
    }
    const int node_num = (int)order.size();
    std::vector<int> next((size_t)node_num, node_num);
    {
        std::vector<int> st{0};
        int k = 0;
        while (!st.empty()) {
            const int cur = st.back();
            st.pop_back();
            next[(size_t)k] = st.empty() ? node_num : tindex[(size_t)st.back()];
            const GNode& g = nodes[(size_t)cur];
            if (g.right != -1) st.push_back(g.right);
            if (g.left != -1) st.push_back(g.left);
            k++;
        }
    }
    int leaves = 0;
    for (int id : order) leaves += nodes[(size_t)id].leaf ? 1 : 0;
    pt_bvh_node_device* out = (pt_bvh_node_device*)std::calloc((size_t)node_num, sizeof(pt_bvh_node_device));
    int* slots = (int*)std::malloc((size_t)std::max(leaves, 1) * (size_t)leaf_size * sizeof(int));
    if (!out || !slots) { std::free(out); std::free(slots); return -2; }
    int li = 0;
    for (int k = 0; k < node_num; k++) {
        const GNode& g = nodes[(size_t)order[(size_t)k]];
        pt_bvh_node_device& d = out[k];
        d.box.left_bottom = {g.box.lb[0], g.box.lb[1], g.box.lb[2]};
        d.box.right_top = {g.box.rt[0], g.box.rt[1], g.box.rt[2]};
        d.box.centroid = {0.5f * (g.box.rt[0] + g.box.lb[0]), 0.5f * (g.box.rt[1] + g.box.lb[1]),
                          0.5f * (g.box.rt[2] + g.box.lb[2])};
        d.is_leaf = g.leaf ? 1 : 0;
        d.next_node_index = next[(size_t)k];
        d.triangle_indices = nullptr;
        if (g.leaf) {
            for (int j = 0; j < leaf_size; j++) slots[(size_t)li * leaf_size + j] = j < (int)g.tris.size() ? g.tris[(size_t)j] : -1;
            d.triangle_indices = slots + (size_t)li * leaf_size;
            li++;
        }
    }
    *nodes_out = out;
    *node_num_out = node_num;
    *leaf_out = slots;
    *leaf_num_out = li;
    return 0;
}

}  // namespace

int pt_flatten_tree(std::vector<PtTreeNode>& nodes, int leaf_size, pt_bvh_node_device** nodes_out, int* node_num_out,
                    int** leaf_out, int* leaf_num_out) {
    return flatten_tree(nodes, leaf_size, nodes_out, node_num_out, leaf_out, leaf_num_out);
}

// bvh_naive_cpu::build_bvh (Bvh/bvh.cpp:185-219) + build_bvh_device_data (:244-330).
extern "C" int pt_bvh_build_naive(const pt_triangle* tris, int n, int start_index, int leaf_size, int bucket_num,
                                  pt_bvh_node_device** nodes_out, int* node_num_out, int** leaf_out, int* leaf_num_out) {
    if (!tris || n <= 0 || leaf_size <= 0 || bucket_num <= 0 || !nodes_out || !node_num_out || !leaf_out || !leaf_num_out)
        return -1;
    std::vector<GNode> nodes(1);
    GNode& root = nodes[0];
    root.box = box_of_triangle(tris[0]);
    std::vector<Box> boxes((size_t)n);
    for (int i = 0; i < n; i++) {
        boxes[(size_t)i] = box_of_triangle(tris[i]);
        expand(root.box, boxes[(size_t)i]);  // expand_to_fit_triangle
        root.tris.push_back(i + start_index);
    }
    if ((int)root.tris.size() <= leaf_size) {
        root.leaf = true;
    } else {
        naive_split(nodes, boxes, start_index, leaf_size, bucket_num);
    }
    return flatten_tree(nodes, leaf_size, nodes_out, node_num_out, leaf_out, leaf_num_out);
}

// ---- PT_BVH_SAH: a binned surface-area-heuristic tree (not a reference builder) ------------------------------------
// The reference's trees are its Morton LBVH (config default MortonCodeCUDA, Bvh/bvh.cpp:862-1047) and a bucketed
// split priced by 2 * VOLUME (bounding_box.h:63-66, bvh.cpp:117). This one prices splits by true surface area
// (MacDonald & Booth): per node, the triangle centroids binned along each axis (`bins` equal bins over the centroid
// extent), the split minimising SA(left) * n(left) + SA(right) * n(right), leaves of at most `leaf_size` triangles
// (one triangle per leaf at the reference's BvhLeafNodeTriangleNum = 1). The tree is flattened exactly as the
// reference flattens its own (flatten_tree: preorder, skip indices, thin leaf boxes widened to the parent's), so the
// walk (path_tracer_kernel.cu:111-150) and every kernel run on it unchanged; the closest hit differs from the
// reference tree's only where the walk order decides it (ties, boxes grazed in float), DESIGN.md §5.
// Preorder child order (PT_SAH_ORDER, the study's knob): 0 the lower side of the split first, 1 the child of larger
// surface area first, 2 the child with more triangles first, 3 the smaller surface area first, 4 fewer triangles first,
// 5 the upper side first, 6 (default) the order of least expected dependent steps (pt_sah_order_by_steps). Orders
// 1-6 visit about the same nodes (metric -8 %, C4 -14 % against the reference tree), but the GPU walk is bound by its
// dependent steps, and those differ: per mesh walk on the metric frame the reference tree takes 5.16, order 2 5.44,
// order 6 4.72 (C4: 9.10, 8.62, 7.77; tools/traversal_study.py, profiles/r06/tree/).
int pt_sah_bins() {  // centroid bins per axis (PT_SAH_BINS, the study's knob; 2..64)
    const char* e = std::getenv("PT_SAH_BINS");
    const int b = e ? std::atoi(e) : 32;
    return b < 2 ? 2 : (b > 64 ? 64 : b);
}

int pt_sah_order() {
    const char* e = std::getenv("PT_SAH_ORDER");
    return e ? std::atoi(e) : 6;
}

namespace {

inline double sa_of(const Box& b) {
    const double x = (double)b.rt[0] - b.lb[0], y = (double)b.rt[1] - b.lb[1], z = (double)b.rt[2] - b.lb[2];
    return 2.0 * (x * y + y * z + z * x);
}

int sah_build(const pt_triangle* tris, int n, int start, int leaf_size, int bins, std::vector<GNode>& nodes) {
    const int order = pt_sah_order() == 6 ? 0 : pt_sah_order();  // 6: reordered afterwards (pt_sah_order_by_steps)
    bins = std::max(2, std::min(bins, 256));
    std::vector<Box> box((size_t)n);
    std::vector<float> cen((size_t)n * 3);
    for (int i = 0; i < n; i++) {
        box[(size_t)i] = box_of_triangle(tris[i]);
        ptbvh::canonical_zeros(box[(size_t)i]);  // the device builder's unions are order-free (pt_bvh_sah.hip)
        for (int k = 0; k < 3; k++) cen[(size_t)i * 3 + k] = 0.5f * (box[(size_t)i].lb[k] + box[(size_t)i].rt[k]);
    }
    std::vector<int> idx((size_t)n);
    for (int i = 0; i < n; i++) idx[(size_t)i] = i;
    struct Task { int node, begin, end; };
    nodes.assign(1, GNode{});
    std::vector<Task> stack{{0, 0, n}};
    std::vector<Box> bbox((size_t)bins);
    std::vector<int> bcnt((size_t)bins);
    std::vector<char> binit((size_t)bins);
    std::vector<double> right_sa((size_t)bins);
    std::vector<int> right_n((size_t)bins);
    while (!stack.empty()) {
        const Task t = stack.back();
        stack.pop_back();
        const int cnt = t.end - t.begin;
        Box nb = box[(size_t)idx[(size_t)t.begin]];
        float clo[3], chi[3];
        for (int k = 0; k < 3; k++) clo[k] = chi[k] = cen[(size_t)idx[(size_t)t.begin] * 3 + k];
        for (int i = t.begin + 1; i < t.end; i++) {
            const int j = idx[(size_t)i];
            expand(nb, box[(size_t)j]);
            for (int k = 0; k < 3; k++) {
                clo[k] = std::min(clo[k], cen[(size_t)j * 3 + k]);
                chi[k] = std::max(chi[k], cen[(size_t)j * 3 + k]);
            }
        }
        nodes[(size_t)t.node].box = nb;
        if (cnt <= leaf_size) {
            GNode& g = nodes[(size_t)t.node];
            g.leaf = true;
            g.tris.assign((size_t)leaf_size, -1);
            for (int i = 0; i < cnt; i++) g.tris[(size_t)i] = idx[(size_t)(t.begin + i)] + start;
            continue;
        }
        double best = INFINITY;
        int best_axis = -1, best_bin = 0;
        for (int k = 0; k < 3; k++) {
            const float ext = chi[k] - clo[k];
            if (!(ext > 0.0f)) continue;
            const float scale = (float)bins / ext;
            std::fill(bcnt.begin(), bcnt.end(), 0);
            std::fill(binit.begin(), binit.end(), 0);
            for (int i = t.begin; i < t.end; i++) {
                const int j = idx[(size_t)i];
                const int b = std::min(bins - 1, (int)((cen[(size_t)j * 3 + k] - clo[k]) * scale));
                if (!binit[(size_t)b]) { bbox[(size_t)b] = box[(size_t)j]; binit[(size_t)b] = 1; }
                else expand(bbox[(size_t)b], box[(size_t)j]);
                bcnt[(size_t)b]++;
            }
            Box acc{};
            bool any = false;
            int nr = 0;
            for (int b = bins - 1; b >= 1; b--) {  // right side = bins [b, bins)
                if (binit[(size_t)b]) { if (!any) { acc = bbox[(size_t)b]; any = true; } else expand(acc, bbox[(size_t)b]); }
                nr += bcnt[(size_t)b];
                right_sa[(size_t)b] = any ? sa_of(acc) : 0.0;
                right_n[(size_t)b] = nr;
            }
            any = false;
            int nl = 0;
            for (int b = 1; b < bins; b++) {  // left side = bins [0, b)
                if (binit[(size_t)(b - 1)]) {
                    if (!any) { acc = bbox[(size_t)(b - 1)]; any = true; } else expand(acc, bbox[(size_t)(b - 1)]);
                }
                nl += bcnt[(size_t)(b - 1)];
                if (nl == 0 || right_n[(size_t)b] == 0) continue;
                const double c = sa_of(acc) * nl + right_sa[(size_t)b] * right_n[(size_t)b];
                if (c < best) { best = c; best_axis = k; best_bin = b; }
            }
        }
        int mid;
        if (best_axis < 0) {  // every centroid the same: split the range in half
            mid = t.begin + cnt / 2;
        } else {
            const float scale = (float)bins / (chi[best_axis] - clo[best_axis]);
            const auto it = std::stable_partition(idx.begin() + t.begin, idx.begin() + t.end, [&](int j) {
                return std::min(bins - 1, (int)((cen[(size_t)j * 3 + best_axis] - clo[best_axis]) * scale)) < best_bin;
            });
            mid = (int)(it - idx.begin());
        }
        const int l = (int)nodes.size(), r = l + 1;
        nodes.emplace_back();
        nodes.emplace_back();
        nodes[(size_t)l].parent = nodes[(size_t)r].parent = t.node;
        int first = l, second = r;  // preorder: `first` is walked first
        if (order != 0) {
            Box bl = box[(size_t)idx[(size_t)t.begin]], br = box[(size_t)idx[(size_t)mid]];
            for (int i = t.begin + 1; i < mid; i++) expand(bl, box[(size_t)idx[(size_t)i]]);
            for (int i = mid + 1; i < t.end; i++) expand(br, box[(size_t)idx[(size_t)i]]);
            const double sl = sa_of(bl), sr = sa_of(br);
            const int nl = mid - t.begin, nr = t.end - mid;
            const bool swap = order == 1 ? sr > sl : order == 2 ? nr > nl : order == 3 ? sr < sl : order == 4 ? nr < nl
                                                                                      : true;  // 5: upper side first
            if (swap) std::swap(first, second);
        }
        nodes[(size_t)t.node].left = first;
        nodes[(size_t)t.node].right = second;
        stack.push_back({r, mid, t.end});
        stack.push_back({l, t.begin, mid});
    }
    return 0;
}

}  // namespace

// Child order 6: the order that minimises the walk's expected dependent steps (pass_kernel_u's two-record step,
// pt_path.h walk_box_inline), bottom-up. A step loads the records at pos and pos + 1, so a passing internal node's
// first child is tested in the same step ("free") while its second child is reached by a skip and starts a step of its
// own. With P(Y) = SA(Y) / SA(parent) the chance that a ray through the parent passes Y (1 for a thin leaf, whose box
// the flattening widens to its parent's):
//   start(leaf) = 1,  free(leaf) = P                       (a passing second-record leaf is re-tested with its triangle)
//   start(Y) = 1 + P(Y) (free(F) + start(S)),  free(Y) = P(Y) (start(F) + start(S))   for Y's children F first, S second
// and each node takes the order with the smaller free(F) + start(S).
void pt_sah_order_by_steps(std::vector<PtTreeNode>& nodes) {
    if (nodes.empty()) return;
    std::vector<int> post;
    post.reserve(nodes.size());
    {
        std::vector<std::pair<int, int>> st{{0, 0}};
        while (!st.empty()) {
            auto& top = st.back();
            const PtTreeNode& g = nodes[(size_t)top.first];
            if (!g.leaf && top.second < 2) {
                const int c = top.second++ == 0 ? g.left : g.right;
                st.push_back({c, 0});
                continue;
            }
            post.push_back(top.first);
            st.pop_back();
        }
    }
    std::vector<double> cstart(nodes.size(), 1.0), cfree(nodes.size(), 0.0), prob(nodes.size(), 1.0);
    for (size_t i = 0; i < nodes.size(); i++) {
        const PtTreeNode& g = nodes[i];
        if (g.leaf || g.left < 0) continue;
        const double sp = sa_of(g.box);
        for (int c : {g.left, g.right}) {
            const PtTreeNode& k = nodes[(size_t)c];
            prob[(size_t)c] = (k.leaf && is_thin(k.box)) || !(sp > 0.0) ? 1.0 : std::min(1.0, sa_of(k.box) / sp);
        }
    }
    for (int id : post) {
        PtTreeNode& g = nodes[(size_t)id];
        if (g.leaf) {
            cstart[(size_t)id] = 1.0;
            cfree[(size_t)id] = prob[(size_t)id];
            continue;
        }
        const int a = g.left, b = g.right;
        const double ab = cfree[(size_t)a] + cstart[(size_t)b], ba = cfree[(size_t)b] + cstart[(size_t)a];
        if (ba < ab) std::swap(g.left, g.right);
        cstart[(size_t)id] = 1.0 + prob[(size_t)id] * std::min(ab, ba);
        cfree[(size_t)id] = prob[(size_t)id] * (cstart[(size_t)a] + cstart[(size_t)b]);
    }
}

// Treelet restructuring (Karras & Aila 2013, "Fast parallel construction of high-quality BVHs"), the study's knob
// PT_SAH_TREELET = k (treelet leaves, 3..8; 0 off): every internal node, children first, becomes the root of a
// treelet grown by opening its largest-area treelet leaf until k leaves; the treelet's topology is rebuilt as the one
// of least total internal surface area (dynamic programming over the 2^k leaf subsets), reusing its internal nodes.
void pt_treelet_restructure(std::vector<PtTreeNode>& nodes, int k) {
    if (k < 3 || nodes.size() < 3) return;
    k = std::min(k, 8);
    std::vector<int> post;
    {
        std::vector<std::pair<int, int>> st{{0, 0}};
        while (!st.empty()) {
            auto& top = st.back();
            const PtTreeNode& g = nodes[(size_t)top.first];
            if (!g.leaf && top.second < 2) {
                const int c = top.second++ == 0 ? g.left : g.right;
                st.push_back({c, 0});
                continue;
            }
            post.push_back(top.first);
            st.pop_back();
        }
    }
    const int full = 1 << k;
    std::vector<Box> ubox((size_t)full);
    std::vector<double> best((size_t)full);
    std::vector<int> split((size_t)full);
    for (int root : post) {
        if (nodes[(size_t)root].leaf) continue;
        std::vector<int> L{nodes[(size_t)root].left, nodes[(size_t)root].right}, I{root};
        while ((int)L.size() < k) {
            int pick = -1;
            double area = -1.0;
            for (int i = 0; i < (int)L.size(); i++) {
                const PtTreeNode& g = nodes[(size_t)L[(size_t)i]];
                if (g.leaf) continue;
                const double a = sa_of(g.box);
                if (a > area) { area = a; pick = i; }
            }
            if (pick < 0) break;
            const int id = L[(size_t)pick];
            L.erase(L.begin() + pick);
            L.push_back(nodes[(size_t)id].left);
            L.push_back(nodes[(size_t)id].right);
            I.push_back(id);
        }
        const int n = (int)L.size();
        if (n < 3) continue;
        const int all = (1 << n) - 1;
        for (int S = 1; S <= all; S++) {
            const int low = __builtin_ctz((unsigned)S);
            const int rest = S & (S - 1);
            ubox[(size_t)S] = nodes[(size_t)L[(size_t)low]].box;
            if (rest) expand(ubox[(size_t)S], ubox[(size_t)rest]);
            if (!rest) { best[(size_t)S] = 0.0; continue; }
            // the partitions {P, S \ P} with P holding S's lowest leaf
            double b = INFINITY;
            int bp = 0;
            const int lowbit = S & -S;
            for (int P = (S - 1) & S; P; P = (P - 1) & S) {
                if (!(P & lowbit)) continue;
                const double c = best[(size_t)P] + best[(size_t)(S ^ P)];
                if (c < b) { b = c; bp = P; }
            }
            best[(size_t)S] = b + sa_of(ubox[(size_t)S]);
            split[(size_t)S] = bp;
        }
        // rebuild: subset `all` at `root`, the internal nodes of the other subsets in the freed slots
        size_t next_slot = 1;
        std::vector<std::pair<int, int>> work{{all, root}};
        while (!work.empty()) {
            const auto [S, id] = work.back();
            work.pop_back();
            PtTreeNode& g = nodes[(size_t)id];
            g.box = ubox[(size_t)S];
            g.leaf = false;
            const int P = split[(size_t)S], Q = S ^ P;
            int child[2];
            int sub[2] = {P, Q};
            for (int side = 0; side < 2; side++) {
                if ((sub[side] & (sub[side] - 1)) == 0) {
                    child[side] = L[(size_t)__builtin_ctz((unsigned)sub[side])];
                } else {
                    child[side] = I[next_slot++];
                    work.push_back({sub[side], child[side]});
                }
                nodes[(size_t)child[side]].parent = id;
            }
            g.left = child[0];
            g.right = child[1];
        }
    }
}

extern "C" int pt_bvh_build_sah(const pt_triangle* tris, int n, int start_index, int leaf_size, int bins,
                                pt_bvh_node_device** nodes_out, int* node_num_out, int** leaf_out, int* leaf_num_out) {
    if (!tris || n <= 0 || leaf_size <= 0 || bins <= 0 || !nodes_out || !node_num_out || !leaf_out || !leaf_num_out)
        return -1;
    std::vector<GNode> nodes;
    int rc = sah_build(tris, n, start_index, leaf_size, bins, nodes);
    if (rc != 0) return rc;
    if (const char* e = std::getenv("PT_SAH_TREELET")) pt_treelet_restructure(nodes, std::atoi(e));
    if (pt_sah_order() == 6) pt_sah_order_by_steps(nodes);
    return flatten_tree(nodes, leaf_size, nodes_out, node_num_out, leaf_out, leaf_num_out);
}

extern "C" int pt_bvh_build_ex(const pt_triangle* tris, int n, int start_index, int leaf_size, int method, int bucket_num,
                               pt_bvh_node_device** nodes_out, int* node_num_out, int** leaf_out, int* leaf_num_out) {
    if (method == PT_BVH_NAIVE_CPU)
        return pt_bvh_build_naive(tris, n, start_index, leaf_size, bucket_num, nodes_out, node_num_out, leaf_out, leaf_num_out);
    if (method == PT_BVH_SAH)
        return pt_bvh_build_sah(tris, n, start_index, leaf_size, pt_sah_bins(), nodes_out, node_num_out, leaf_out,
                                leaf_num_out);
    // MortonCodeCPU and MortonCodeCUDA build the same tree (Bvh/bvh.cpp:667-780 vs :862-1047); the
    // CPU variant's std::sort is not stable, so equal codes keep their input order here as in the
    // CUDA variant's merge sort.
    const int rc = pt_bvh_build(tris, n, start_index, leaf_size, method, nodes_out, node_num_out, leaf_out, leaf_num_out);
    // the tree study's "LBVH + treelet restructuring" (PT_LBVH_TREELET = k, off by default; never the reference
    // tree): the flattened Morton tree read back into a linked tree, restructured, flattened again
    const char* tl = std::getenv("PT_LBVH_TREELET");
    if (rc != 0 || !tl || std::atoi(tl) < 3) return rc;
    const pt_bvh_node_device* fl = *nodes_out;
    const int nn = *node_num_out;
    std::vector<GNode> g((size_t)nn);
    for (int i = 0; i < nn; i++) {
        g[(size_t)i].box = Box{{fl[i].box.left_bottom.x, fl[i].box.left_bottom.y, fl[i].box.left_bottom.z},
                               {fl[i].box.right_top.x, fl[i].box.right_top.y, fl[i].box.right_top.z}};
        g[(size_t)i].leaf = fl[i].is_leaf != 0;
        if (g[(size_t)i].leaf) {
            g[(size_t)i].tris.assign(fl[i].triangle_indices, fl[i].triangle_indices + leaf_size);
        } else {
            g[(size_t)i].left = i + 1;
            g[(size_t)i].right = fl[i + 1].next_node_index;
            g[(size_t)(i + 1)].parent = g[(size_t)fl[i + 1].next_node_index].parent = i;
        }
    }
    pt_bvh_free(*nodes_out, *leaf_out);
    pt_treelet_restructure(g, std::atoi(tl));
    if (pt_sah_order() == 6) pt_sah_order_by_steps(g);
    return flatten_tree(g, leaf_size, nodes_out, node_num_out, leaf_out, leaf_num_out);
}

// ---- scene assembly ----------------------------------------------------------------------------
struct pt_scene_builder {
    std::vector<pt_material> materials;
    std::vector<pt_sphere> spheres;
    std::vector<pt_triangle> triangles;
    std::vector<int> tri_material;
    std::vector<int> mesh_start, mesh_count;
    // the interactive-edit state of Core/triangle_mesh.h: mesh-local triangles (m_triangles: loaded and
    // rotated, before translate * scale), position / scale / rotate and the rotation already applied,
    // the inverse of the transform the BVH was built under (m_mesh_initial_transform) and the boxes of
    // that build (m_mesh_bvh_initial_device)
    std::vector<pt_triangle> local;
    std::vector<pt_float3> mesh_pos, mesh_scl, mesh_rot, mesh_rot_applied;
    std::vector<ptglm::M4> init_inv;
    std::vector<pt_float3> init_pos, init_scl;  // the transform init_inv inverts
    std::vector<std::vector<pt_bounding_box>> init_boxes;
    int build_leaf = 1, build_method = 2, build_bucket = 12;
    std::vector<std::vector<unsigned char>> textures;
    std::vector<int> tex_w, tex_h;
    std::vector<unsigned char> cube;
    int cube_len = 0;
    // built state
    std::vector<pt_bvh_node_device*> bvh_nodes;
    std::vector<int*> bvh_leaf;
    std::vector<int> node_num;
    std::vector<pt_texture_wrapper> tex_wrappers;
    pt_cube_map cube_map{};
    bool built = false;
    int bvh_device = -2;  // MortonCodeCUDA builds on: -2 the HIP device when one is present, -1 the host, >= 0 the device

    void release_bvh() {
        for (size_t i = 0; i < bvh_nodes.size(); i++) pt_bvh_free(bvh_nodes[i], bvh_leaf[i]);
        bvh_nodes.clear(); bvh_leaf.clear(); node_num.clear();
        built = false;
    }
    ~pt_scene_builder() { release_bvh(); }
};

extern "C" pt_scene_builder* pt_scene_builder_create(void) { return new pt_scene_builder(); }
extern "C" void pt_scene_builder_destroy(pt_scene_builder* b) { delete b; }

extern "C" int pt_scene_builder_add_material(pt_scene_builder* b, const pt_material* m) {
    if (!b || !m) return -1;
    b->materials.push_back(*m);
    b->built = false;
    return (int)b->materials.size() - 1;
}

extern "C" int pt_scene_builder_add_sphere(pt_scene_builder* b, pt_float3 center, float radius, const pt_material* m) {
    if (!b || !m) return -1;
    pt_sphere s;
    std::memset(&s, 0, sizeof(s));
    s.center = center;
    s.radius = radius;
    s.mat = *m;
    b->spheres.push_back(s);
    return (int)b->spheres.size() - 1;
}

namespace {
using namespace ptglm;

// glm::rotate (glm/gtc/matrix_transform.inl:18-47) about a unit coordinate axis (host libm cos/sin, as
// the reference's host code)
M4 rotate4(const M4& m, float angle, int axis_index) {
    const float c = std::cos(angle), s = std::sin(angle);
    float axis[3] = {0.0f, 0.0f, 0.0f};
    axis[axis_index] = 1.0f;  // normalize() of a unit axis is exact
    const float temp[3] = {(1.0f - c) * axis[0], (1.0f - c) * axis[1], (1.0f - c) * axis[2]};
    float R[3][3];
    R[0][0] = c + temp[0] * axis[0];
    R[0][1] = temp[0] * axis[1] + s * axis[2];
    R[0][2] = temp[0] * axis[2] - s * axis[1];
    R[1][0] = temp[1] * axis[0] - s * axis[2];
    R[1][1] = c + temp[1] * axis[1];
    R[1][2] = temp[1] * axis[2] + s * axis[0];
    R[2][0] = temp[2] * axis[0] + s * axis[1];
    R[2][1] = temp[2] * axis[1] - s * axis[0];
    R[2][2] = c + temp[2] * axis[2];
    M4 r;
    for (int i = 0; i < 3; i++)
        set_col(r, i, add4(add4(mul4(col(m, 0), R[i][0]), mul4(col(m, 1), R[i][1])), mul4(col(m, 2), R[i][2])));
    set_col(r, 3, col(m, 3));
    return r;
}

inline pt_float3 normalize_host(float x, float y, float z) {
    float o[3];
    normalize3(x, y, z, o);
    return {o[0], o[1], o[2]};
}
}  // namespace

// triangle_mesh::load_obj (:139-166): rotate Z, then Y, then X (glm::radians degrees), normals by the
// inverse transpose, renormalised; then create_mesh_device_data (:625-647): translate * scale, normals
// by its inverse transpose, renormalised.
extern "C" int pt_scene_builder_add_mesh(pt_scene_builder* b, int tri_num, const float* v, const float* nrm,
                                         const float* uv, const int* tri_material, pt_float3 pos, pt_float3 scl,
                                         pt_float3 rot) {
    if (!b || tri_num <= 0 || !v || !nrm || !tri_material) return -1;
    const float deg = 0.01745329251994329576923690768489f;  // glm::radians
    M4 R = identity4();
    R = rotate4(R, rot.z * deg, 2);
    R = rotate4(R, rot.y * deg, 1);
    R = rotate4(R, rot.x * deg, 0);
    const M4 Rn = transpose4(inverse4(R));
    M4 T = identity4();  // glm::translate(I, pos) then glm::scale(., scl)
    set_col(T, 3, add4(add4(add4(mul4(col(T, 0), pos.x), mul4(col(T, 1), pos.y)), mul4(col(T, 2), pos.z)), col(T, 3)));
    set_col(T, 0, mul4(col(T, 0), scl.x));
    set_col(T, 1, mul4(col(T, 1), scl.y));
    set_col(T, 2, mul4(col(T, 2), scl.z));
    const M4 Tn = transpose4(inverse4(T));
    b->mesh_start.push_back((int)b->triangles.size());
    b->mesh_count.push_back(tri_num);
    b->mesh_pos.push_back(pos);
    b->mesh_scl.push_back(scl);
    b->mesh_rot.push_back(rot);
    b->mesh_rot_applied.push_back(rot);
    b->init_inv.push_back(inverse4(T));
    b->init_pos.push_back(pos);
    b->init_scl.push_back(scl);
    b->init_boxes.emplace_back();
    for (int t = 0; t < tri_num; t++) {
        pt_triangle tr, lt;
        std::memset(&tr, 0, sizeof(tr));
        std::memset(&lt, 0, sizeof(lt));
        pt_float3* vo[3] = {&tr.vertex0, &tr.vertex1, &tr.vertex2};
        pt_float3* no[3] = {&tr.normal0, &tr.normal1, &tr.normal2};
        pt_float2* uo[3] = {&tr.uv0, &tr.uv1, &tr.uv2};
        for (int k = 0; k < 3; k++) {
            const float* p = v + (size_t)t * 9 + k * 3;
            const float* q = nrm + (size_t)t * 9 + k * 3;
            const V4 rv = mat_vec(R, V4{p[0], p[1], p[2], 1.0f});
            const V4 rn = mat_vec(Rn, V4{q[0], q[1], q[2], 0.0f});
            const pt_float3 n1 = normalize_host(rn.x, rn.y, rn.z);
            const V4 wv = mat_vec(T, V4{rv.x, rv.y, rv.z, 1.0f});
            const V4 wn = mat_vec(Tn, V4{n1.x, n1.y, n1.z, 0.0f});
            *vo[k] = {wv.x, wv.y, wv.z};
            *no[k] = normalize_host(wn.x, wn.y, wn.z);
            (&lt.vertex0)[k] = {rv.x, rv.y, rv.z};
            (&lt.normal0)[k] = n1;
            if (uv) *uo[k] = {uv[(size_t)t * 6 + k * 2], uv[(size_t)t * 6 + k * 2 + 1]};
            else *uo[k] = {0.0f, 0.0f};
        }
        b->triangles.push_back(tr);
        b->local.push_back(lt);
        b->tri_material.push_back(tri_material[t]);
    }
    b->built = false;
    return (int)b->mesh_start.size() - 1;
}

extern "C" int pt_scene_builder_set_cube_map(pt_scene_builder* b, int length, const unsigned char* faces) {
    if (!b || length <= 0 || !faces) return -1;
    b->cube.assign(faces, faces + (size_t)6 * length * length * 4);
    b->cube_len = length;
    b->built = false;
    return 0;
}

extern "C" int pt_scene_builder_add_texture(pt_scene_builder* b, int w, int h, const unsigned char* rgba) {
    if (!b || w <= 0 || h <= 0 || !rgba) return -1;
    b->textures.emplace_back(rgba, rgba + (size_t)w * h * 4);
    b->tex_w.push_back(w);
    b->tex_h.push_back(h);
    b->built = false;
    return (int)b->textures.size() - 1;
}

extern "C" int pt_scene_builder_build(pt_scene_builder* b, int leaf_size, int method) {
    return pt_scene_builder_build_ex(b, leaf_size, method, 12);
}

extern "C" int pt_scene_builder_set_bvh_device(pt_scene_builder* b, int device) {
    if (!b || device < -2) return -1;
    b->bvh_device = device;
    b->built = false;
    return 0;
}

namespace {
// One mesh's BVH with the builder's configured method (MortonCodeCUDA on the GPU when present).
int build_mesh_bvh(pt_scene_builder* b, size_t m, pt_bvh_node_device** nodes, int* nn, int** leaf, int* ln) {
    // MortonCodeCUDA runs on the GPU (pt_bvh.hip); its node array equals the host builder's bit for bit
    // (tests/test_bvh_device.py), which therefore serves machines without a HIP device
    // PT_BVH_SAH likewise (pt_bvh_sah.hip, the host builder's tree byte for byte) for meshes large enough to pay for
    // the launches
    const bool device = b->bvh_device >= 0 || (b->bvh_device == -2 && pt_device_count() > 0);
    const pt_triangle* t = b->triangles.data() + b->mesh_start[m];
    if (device && b->build_method == PT_BVH_MORTON_CODE_CUDA)
        return pt_bvh_build_device(t, b->mesh_count[m], b->mesh_start[m], b->build_leaf, nodes, nn, leaf, ln);
    if (device && b->build_method == PT_BVH_SAH && b->mesh_count[m] >= 4096)
        return pt_bvh_build_sah_device(t, b->mesh_count[m], b->mesh_start[m], b->build_leaf, pt_sah_bins(), nodes, nn,
                                       leaf, ln);
    return pt_bvh_build_ex(t, b->mesh_count[m], b->mesh_start[m], b->build_leaf, b->build_method, b->build_bucket,
                           nodes, nn, leaf, ln);
}

// The boxes of a fresh build are the mesh's initial boxes, under its current transform
// (Core/triangle_mesh.cpp:498-540 keeps the first device copy as m_mesh_bvh_initial_device).
void snapshot_initial(pt_scene_builder* b, size_t m) {
    const pt_bvh_node_device* nodes = b->bvh_nodes[m];
    b->init_boxes[m].resize((size_t)b->node_num[m]);
    for (int i = 0; i < b->node_num[m]; i++) b->init_boxes[m][i] = nodes[i].box;
    const pt_float3 p = b->mesh_pos[m], s = b->mesh_scl[m];
    b->init_inv[m] = inverse4(translate_scale(p.x, p.y, p.z, s.x, s.y, s.z));
    b->init_pos[m] = p;
    b->init_scl[m] = s;
}
}  // namespace

extern "C" int pt_scene_builder_build_ex(pt_scene_builder* b, int leaf_size, int method, int bucket_num) {
    if (!b) return -1;
    b->release_bvh();
    for (size_t t = 0; t < b->triangles.size(); t++) {
        int m = b->tri_material[t];
        if (m < 0 || m >= (int)b->materials.size()) return -3;
        b->triangles[t].mat = b->materials.data() + m;
    }
    b->build_leaf = leaf_size;
    b->build_method = method;
    b->build_bucket = bucket_num;
    for (size_t m = 0; m < b->mesh_start.size(); m++) {
        pt_bvh_node_device* nodes = nullptr;
        int nn = 0, *leaf = nullptr, ln = 0;
        int rc = build_mesh_bvh(b, m, &nodes, &nn, &leaf, &ln);
        if (rc != 0) return rc;
        b->bvh_nodes.push_back(nodes);
        b->bvh_leaf.push_back(leaf);
        b->node_num.push_back(nn);
        snapshot_initial(b, m);
    }
    b->tex_wrappers.clear();
    for (size_t i = 0; i < b->textures.size(); i++)
        b->tex_wrappers.push_back({b->tex_w[i], b->tex_h[i], b->textures[i].data()});
    if (b->cube_len > 0) {
        size_t face = (size_t)b->cube_len * b->cube_len * 4;
        unsigned char* base = b->cube.data();
        b->cube_map = {base, base + face, base + 2 * face, base + 3 * face, base + 4 * face, base + 5 * face, b->cube_len};
    }
    b->built = true;
    return 0;
}

// triangle_mesh::set_transform_device (Core/triangle_mesh.cpp:271-328) with bvh_update_function = update_bvh
// (Bvh/bvh.cpp:332-356): the mesh's triangles become translate(position) * scale(scale) applied to its
// mesh-local triangles (normals by the inverse transpose, renormalised); every node box becomes
// (transform * initial_transform) applied to its two corners in the initial build, centroid = their mean.
extern "C" int pt_scene_builder_set_transform(pt_scene_builder* b, int mesh, pt_float3 position, pt_float3 scale) {
    if (!b || !b->built || mesh < 0 || mesh >= (int)b->mesh_start.size()) return -1;
    const M4 T = translate_scale(position.x, position.y, position.z, scale.x, scale.y, scale.z);
    const M4 Tn = transpose4(inverse4(T));
    b->mesh_pos[mesh] = position;
    b->mesh_scl[mesh] = scale;
    for (int t = b->mesh_start[mesh]; t < b->mesh_start[mesh] + b->mesh_count[mesh]; t++) {
        const pt_triangle& lt = b->local[t];
        pt_triangle& tr = b->triangles[t];
        for (int k = 0; k < 3; k++) {
            const pt_float3 v = (&lt.vertex0)[k], n = (&lt.normal0)[k];
            const V4 wv = mat_vec(T, V4{v.x, v.y, v.z, 1.0f});
            const V4 wn = mat_vec(Tn, V4{n.x, n.y, n.z, 0.0f});
            (&tr.vertex0)[k] = {wv.x, wv.y, wv.z};
            (&tr.normal0)[k] = normalize_host(wn.x, wn.y, wn.z);
        }
    }
    const M4 C = mat_mul(T, b->init_inv[mesh]);  // transform_mat * initial_transform_mat (bvh.cpp:348-349)
    pt_bvh_node_device* nodes = b->bvh_nodes[mesh];
    for (int i = 0; i < b->node_num[mesh]; i++) {
        const pt_bounding_box& ib = b->init_boxes[mesh][i];
        const V4 lb = mat_vec(C, V4{ib.left_bottom.x, ib.left_bottom.y, ib.left_bottom.z, 1.0f});
        const V4 rt = mat_vec(C, V4{ib.right_top.x, ib.right_top.y, ib.right_top.z, 1.0f});
        pt_bounding_box& bx = nodes[i].box;
        bx.left_bottom = {lb.x, lb.y, lb.z};
        bx.right_top = {rt.x, rt.y, rt.z};
        bx.centroid = {0.5f * (lb.x + rt.x), 0.5f * (lb.y + rt.y), 0.5f * (lb.z + rt.z)};
    }
    return 0;
}

// triangle_mesh::set_rotate (:330-333) + apply_rotate (:335-426): the mesh-local triangles are rotated
// by the change of rotation (Z, then Y, then X, in degrees), the mesh is re-transformed, the initial
// transform becomes the inverse of the current one and the mesh's BVH is rebuilt.
extern "C" int pt_scene_builder_set_rotate(pt_scene_builder* b, int mesh, pt_float3 rotate) {
    if (!b || mesh < 0 || mesh >= (int)b->mesh_start.size()) return -1;
    b->mesh_rot[mesh] = rotate;
    return 0;
}

extern "C" int pt_scene_builder_apply_rotate(pt_scene_builder* b, int mesh) {
    if (!b || !b->built || mesh < 0 || mesh >= (int)b->mesh_start.size()) return -1;
    const float deg = 0.01745329251994329576923690768489f;  // glm::radians
    const pt_float3 r = b->mesh_rot[mesh], a = b->mesh_rot_applied[mesh];
    M4 R = identity4();
    R = rotate4(R, (r.z - a.z) * deg, 2);
    R = rotate4(R, (r.y - a.y) * deg, 1);
    R = rotate4(R, (r.x - a.x) * deg, 0);
    const M4 Rn = transpose4(inverse4(R));
    const pt_float3 p = b->mesh_pos[mesh], s = b->mesh_scl[mesh];
    const M4 T = translate_scale(p.x, p.y, p.z, s.x, s.y, s.z);
    const M4 Tn = transpose4(inverse4(T));
    for (int t = b->mesh_start[mesh]; t < b->mesh_start[mesh] + b->mesh_count[mesh]; t++) {
        pt_triangle& lt = b->local[t];
        pt_triangle& tr = b->triangles[t];
        for (int k = 0; k < 3; k++) {
            const pt_float3 v = (&lt.vertex0)[k], n = (&lt.normal0)[k];
            const V4 rv = mat_vec(R, V4{v.x, v.y, v.z, 1.0f});
            const V4 rn = mat_vec(Rn, V4{n.x, n.y, n.z, 0.0f});
            const pt_float3 n1 = normalize_host(rn.x, rn.y, rn.z);
            (&lt.vertex0)[k] = {rv.x, rv.y, rv.z};
            (&lt.normal0)[k] = n1;
            const V4 wv = mat_vec(T, V4{rv.x, rv.y, rv.z, 1.0f});
            const V4 wn = mat_vec(Tn, V4{n1.x, n1.y, n1.z, 0.0f});
            (&tr.vertex0)[k] = {wv.x, wv.y, wv.z};
            (&tr.normal0)[k] = normalize_host(wn.x, wn.y, wn.z);
        }
    }
    pt_bvh_node_device* nodes = nullptr;
    int nn = 0, *leaf = nullptr, ln = 0;
    int rc = build_mesh_bvh(b, (size_t)mesh, &nodes, &nn, &leaf, &ln);
    if (rc != 0) return rc;
    pt_bvh_free(b->bvh_nodes[mesh], b->bvh_leaf[mesh]);
    b->bvh_nodes[mesh] = nodes;
    b->bvh_leaf[mesh] = leaf;
    b->node_num[mesh] = nn;
    snapshot_initial(b, (size_t)mesh);
    b->mesh_rot_applied[mesh] = b->mesh_rot[mesh];
    return 0;
}

// What a device context needs to refit one mesh itself (pt_mesh_attach): its mesh-local triangles,
// where they start in the triangle array, the boxes of its last build and the transform (position,
// scale) that build was made under.
extern "C" int pt_scene_builder_mesh_local(pt_scene_builder* b, int mesh, const pt_triangle** local, int* tri_start,
                                           int* tri_count, const pt_bounding_box** init_boxes, int* node_count,
                                           pt_float3* init_position, pt_float3* init_scale) {
    if (!b || !b->built || mesh < 0 || mesh >= (int)b->mesh_start.size()) return -1;
    if (local) *local = b->local.data() + b->mesh_start[mesh];
    if (tri_start) *tri_start = b->mesh_start[mesh];
    if (tri_count) *tri_count = b->mesh_count[mesh];
    if (init_boxes) *init_boxes = b->init_boxes[mesh].data();
    if (node_count) *node_count = (int)b->init_boxes[mesh].size();
    if (init_position) *init_position = b->init_pos[mesh];
    if (init_scale) *init_scale = b->init_scl[mesh];
    return 0;
}

extern "C" int pt_scene_builder_view(pt_scene_builder* b, pt_scene_view* o) {
    if (!b || !o || !b->built) return -1;
    o->mesh_num = (int)b->bvh_nodes.size();
    o->bvh_nodes = b->bvh_nodes.data();
    o->triangles = b->triangles.data();
    o->triangle_num = (int)b->triangles.size();
    o->sphere_num = (int)b->spheres.size();
    o->spheres = b->spheres.data();
    o->sky_cube_map = b->cube_len > 0 ? &b->cube_map : nullptr;
    o->mesh_textures = b->tex_wrappers.empty() ? nullptr : b->tex_wrappers.data();
    o->texture_num = (int)b->tex_wrappers.size();
    o->materials = b->materials.data();
    o->material_num = (int)b->materials.size();
    o->mesh_node_num = b->node_num.data();
    o->mesh_triangle_start = b->mesh_start.data();
    o->mesh_triangle_num = b->mesh_count.data();
    return 0;
}

// ---- camera (Core/camera.cpp) --------------------------------------------------------------------
extern "C" void pt_view_camera_default(pt_view_camera* c) {
    c->center = {0.0f, 0.0f, 0.0f};
    c->yaw = 0.0f;
    c->pitch = 0.3f;
    c->radius = 14.0f;
    c->aperture_radius = 0.0f;
    c->focal_distance = c->radius;
    c->resolution = {640.0f, 640.0f};
    c->fov = {45.0f, 45.0f};
}

extern "C" void pt_view_camera_set_resolution(pt_view_camera* c, float w, float h) {
    c->resolution = {w, h};
}

extern "C" void pt_view_camera_set_fov(pt_view_camera* c, float fov_x) {
    // math::degrees_to_radians / radians_to_degrees use PI = 3.1415926535897f (basic_math.hpp:14)
    const float PI = 3.1415926535897f;
    c->fov.x = fov_x;
    float half = fov_x / 180.0f * PI * 0.5f;
    c->fov.y = (float)(std::atan(std::tan(half) * (c->resolution.y / c->resolution.x)) * 2.0f) * 180.0f / PI;
}

extern "C" void pt_view_camera_get_render_camera(const pt_view_camera* c, pt_render_camera* r) {
    float x = std::sin(c->yaw) * std::cos(c->pitch);
    float y = std::sin(c->pitch);
    float z = std::cos(c->yaw) * std::cos(c->pitch);
    r->eye = {c->center.x + x * c->radius, c->center.y + y * c->radius, c->center.z + z * c->radius};
    r->view = {-1.0f * x, -1.0f * y, -1.0f * z};
    r->up = {0.0f, 1.0f, 0.0f};
    r->resolution = c->resolution;
    r->fov = c->fov;
    r->focal_distance = c->focal_distance;
    r->aperture_radius = c->aperture_radius;
}

// res/configuration/config.json:1-25 as parsed by config_parser::load_config
extern "C" void pt_configuration_default(pt_configuration* c) {
    std::memset(c, 0, sizeof(*c));
    c->width = 1440;
    c->height = 900;
    c->use_fullscreen = 0;
    c->block_size = 64;
    c->max_block_size = 608;
    c->max_tracer_depth = 20;
    c->vector_bias_length = 0.0002f;
    c->energy_exist_threshold = 0.000001f;
    c->sss_threshold = 0.000001f;
    c->use_sky_box = 1;
    c->use_sky = 0;
    c->use_bilinear = 1;
    c->gamma_correction = 1;
    c->use_anti_alias = 1;
    c->fov = 45.0f;
    c->bvh_leaf_node_triangle_num = 1;
    c->bvh_bucket_max_divide_internal_num = 12;
    c->bvh_build_block_size = 32;
    c->bvh_build = PT_BVH_MORTON_CODE_CUDA;
    c->air_refraction_index = 1.000293f;
    c->air_absorption_coef = {0.0f, 0.0f, 0.0f};
    c->air_reduced_scattering_coef = {0.0f, 0.0f, 0.0f};
    c->cuda_acceleration = 1;
}
