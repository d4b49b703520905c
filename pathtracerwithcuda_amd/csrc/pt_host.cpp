// pt_host.cpp — host-side C++ around the render call: BVH builder, scene assembly in the
// reference data layout, orbit camera, configuration defaults. See include/pt_host.h.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/pt_host.h"

namespace {

// ---- Bvh/bounding_box.h ------------------------------------------------------------------------
struct Box {
    float lb[3], rt[3];
};

inline Box box_of_triangle(const pt_triangle& t) {  // bounding_box::get_bounding_box(v0, v1, v2)
    Box b;
    const float* v0 = &t.vertex0.x;
    const float* v1 = &t.vertex1.x;
    const float* v2 = &t.vertex2.x;
    for (int k = 0; k < 3; k++) {
        float mn = v0[k], mx = v0[k];
        // cuda_math.hpp min(a,b,c) / max(a,b,c): sequential compares
        mn = v1[k] < mn ? v1[k] : mn; mn = v2[k] < mn ? v2[k] : mn;
        mx = v1[k] > mx ? v1[k] : mx; mx = v2[k] > mx ? v2[k] : mx;
        b.lb[k] = mn; b.rt[k] = mx;
    }
    return b;
}

inline void expand(Box& a, const Box& b) {  // expand_to_fit_box: fminf / fmaxf
    for (int k = 0; k < 3; k++) {
        a.lb[k] = std::fmin(a.lb[k], b.lb[k]);
        a.rt[k] = std::fmax(a.rt[k], b.rt[k]);
    }
}

inline bool is_thin(const Box& b) {  // bounding_box::is_thin_bounding_box
    return b.rt[0] == b.lb[0] || b.rt[1] == b.lb[1] || b.rt[2] == b.lb[2];
}

// ---- Bvh/bvh.cpp:370-392 -----------------------------------------------------------------------
inline unsigned int expand_bits(unsigned int v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

inline unsigned int morton(float px, float py, float pz) {
    // fminf(fmaxf(p*1024, 0), 1023): a NaN coordinate (zero mesh extent) maps to 0
    float x = std::fmin(std::fmax(px * 1024.0f, 0.0f), 1023.0f);
    float y = std::fmin(std::fmax(py * 1024.0f, 0.0f), 1023.0f);
    float z = std::fmin(std::fmax(pz * 1024.0f, 0.0f), 1023.0f);
    return expand_bits((unsigned int)x) * 4 + expand_bits((unsigned int)y) * 2 + expand_bits((unsigned int)z);
}

inline unsigned int morton_of_box(const Box& b, const Box& mesh) {
    // (centroid - mesh.lb) / (mesh.rt - mesh.lb), centroid = 0.5 * (rt + lb)
    float c[3], p[3];
    for (int k = 0; k < 3; k++) {
        c[k] = 0.5f * (b.rt[k] + b.lb[k]);
        p[k] = (c[k] - mesh.lb[k]) / (mesh.rt[k] - mesh.lb[k]);
    }
    return morton(p[0], p[1], p[2]);
}

// Bvh/bvh.cpp:398-441 (table-driven; equals __builtin_clz with clz(0) = 32)
inline unsigned int clz32(unsigned int v) { return v == 0 ? 32u : (unsigned int)__builtin_clz(v); }

// Bvh/bvh.cpp:446-481
unsigned int find_split(const std::vector<unsigned int>& code, unsigned int first, unsigned int last) {
    unsigned int fc = code[first], lc = code[last];
    if (fc == lc) return first;
    unsigned int common = clz32(fc ^ lc);
    unsigned int split = first;
    unsigned int step = last - first;
    do {
        step = (step + 1) >> 1;
        unsigned int ns = split + step;
        if (ns < last) {
            if (clz32(fc ^ code[ns]) > common) split = ns;
        }
    } while (step > 1);
    return split;
}

// Bvh/bvh.cpp:486-570, including its unsigned wrap-around and the equal-code run handling.
void find_range(const std::vector<unsigned int>& code, unsigned int n, unsigned int index,
                unsigned int* rx, unsigned int* ry) {
    if (index == 0) { *rx = 0; *ry = n - 1; return; }
    unsigned int initial = index;
    unsigned int prev = code[index - 1], cur = code[index], next = code[index + 1];
    int direction;
    unsigned int delta_min;
    if (prev == cur && cur == next) {
        while (index > 0 && index < n - 1) {
            index++;
            if (index >= n - 1) break;
            if (code[index] != code[index + 1]) break;
        }
        *rx = initial; *ry = index;
        return;
    }
    unsigned int left = clz32(cur ^ prev), right = clz32(cur ^ next);
    if (left > right) { direction = -1; delta_min = right; }
    else { direction = 1; delta_min = left; }
    unsigned int l_max = 2;
    unsigned int test = index + l_max * (unsigned int)direction;
    while (test < n && clz32(cur ^ code[test]) > delta_min) {
        l_max *= 2;
        test = index + l_max * (unsigned int)direction;
    }
    int l = 0;
    for (int divisor = 2; l_max / (unsigned int)divisor >= 1; divisor *= 2) {
        int t = (int)(l_max / (unsigned int)divisor);
        test = index + (unsigned int)((l + t) * direction);
        if (test < n) {
            if (clz32(cur ^ code[test]) > delta_min) l = l + t;
        }
    }
    if (direction == 1) { *rx = index; *ry = index + (unsigned int)(l * direction); }
    else { *rx = index + (unsigned int)(l * direction); *ry = index; }
}

struct BuildNode {
    Box box;
    int left = -1, right = -1;   // child ids: >= 0 internal, <= -2 leaf (-(leaf+2))
    int parent = -1;             // internal id
};

}  // namespace

extern "C" unsigned int pt_morton_code(float x, float y, float z) { return morton(x, y, z); }
extern "C" unsigned int pt_clz_table(unsigned int value) { return clz32(value); }

// bvh_morton_code_cuda::build_bvh (Bvh/bvh.cpp:862-1047) + bvh_naive_cpu::build_bvh_device_data
// (:244-330). thrust::sort with a comparator is a stable merge sort, so std::stable_sort.
extern "C" int pt_bvh_build(const pt_triangle* tris, int n, int start_index, int leaf_size, int method,
                            pt_bvh_node_device** nodes_out, int* node_num_out, int** leaf_out, int* leaf_num_out) {
    (void)method;  // the Morton builder for every method (naive-SAH builder is a later row)
    if (!tris || n <= 0 || leaf_size <= 0 || !nodes_out || !node_num_out || !leaf_out || !leaf_num_out) return -1;

    unsigned int leaf_num = (unsigned int)(n / leaf_size);
    leaf_num = leaf_num == 0 ? 1 : leaf_num;
    leaf_num = (n % leaf_size == 0) ? leaf_num : leaf_num + 1;
    const unsigned int internal_num = leaf_num - 1;

    // mesh box (:889-895)
    Box mesh = box_of_triangle(tris[0]);
    for (int i = 1; i < n; i++) {
        Box b = box_of_triangle(tris[i]);
        expand(mesh, b);
    }

    // per-triangle box + Morton code (bvh_morton_code_kernel.cu:298-326)
    struct TriNode { Box box; unsigned int code; int tri; };
    std::vector<TriNode> tn((size_t)n);
    for (int i = 0; i < n; i++) {
        tn[i].box = box_of_triangle(tris[i]);
        tn[i].code = morton_of_box(tn[i].box, mesh);
        tn[i].tri = i + start_index;
    }
    std::stable_sort(tn.begin(), tn.end(), [](const TriNode& a, const TriNode& b) { return a.code < b.code; });

    // batch into leaves (:920-955), then sort the leaves by the code of their own box
    struct LeafNode { Box box; unsigned int code; int batch; };
    std::vector<LeafNode> leaves(leaf_num);
    std::vector<int> batch_tris((size_t)leaf_num * leaf_size, -1);
    for (unsigned int i = 0; i < leaf_num; i++) {
        int s = (int)i * leaf_size;
        leaves[i].box = tn[s].box;
        batch_tris[(size_t)i * leaf_size] = tn[s].tri;
        for (int j = 1; j < leaf_size; j++) {
            if (j + s < n) {
                expand(leaves[i].box, tn[j + s].box);
                batch_tris[(size_t)i * leaf_size + j] = tn[j + s].tri;
            }
        }
        leaves[i].code = morton_of_box(leaves[i].box, mesh);
        leaves[i].batch = (int)i;
    }
    std::stable_sort(leaves.begin(), leaves.end(), [](const LeafNode& a, const LeafNode& b) { return a.code < b.code; });

    // Karras internal nodes (bvh_morton_code_kernel.cu:262-296), sequential in index order
    std::vector<unsigned int> codes(leaf_num);
    for (unsigned int i = 0; i < leaf_num; i++) codes[i] = leaves[i].code;
    std::vector<BuildNode> inner(internal_num);
    std::vector<int> leaf_parent(leaf_num, -1);
    for (unsigned int i = 0; i < internal_num; i++) {
        unsigned int rx, ry;
        find_range(codes, leaf_num, i, &rx, &ry);
        unsigned int split = find_split(codes, rx, ry);
        if (split == rx) { inner[i].left = -((int)split + 2); leaf_parent[split] = (int)i; }
        else { inner[i].left = (int)split; inner[split].parent = (int)i; }
        if (split + 1 == ry) { inner[i].right = -((int)(split + 1) + 2); leaf_parent[split + 1] = (int)i; }
        else { inner[i].right = (int)(split + 1); inner[split + 1].parent = (int)i; }
    }

    // bottom-up boxes: union of the two children (:817-860), post-order from the root
    auto child_box = [&](int c) -> const Box& { return c <= -2 ? leaves[(size_t)(-c - 2)].box : inner[(size_t)c].box; };
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
    auto node_box = [&](Ref r) -> Box& { return r.leaf ? leaves[(size_t)r.id].box : inner[(size_t)r.id].box; };
    auto parent_of = [&](Ref r) -> int { return r.leaf ? leaf_parent[(size_t)r.id] : inner[(size_t)r.id].parent; };
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
        // traversal index of each (leaf/internal id)
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
                Ref t = st.back();
                next_index[(size_t)k] = t.leaf ? tidx_leaf[(size_t)t.id] : tidx_inner[(size_t)t.id];
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
            int batch = leaves[(size_t)r.id].batch;
            for (int j = 0; j < leaf_size; j++) leaf_idx[(size_t)li * leaf_size + j] = batch_tris[(size_t)batch * leaf_size + j];
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

extern "C" void pt_bvh_free(pt_bvh_node_device* nodes, int* leaf_indices) {
    std::free(nodes);
    std::free(leaf_indices);
}

// ---- scene assembly ----------------------------------------------------------------------------
struct pt_scene_builder {
    std::vector<pt_material> materials;
    std::vector<pt_sphere> spheres;
    std::vector<pt_triangle> triangles;
    std::vector<int> tri_material;
    std::vector<int> mesh_start, mesh_count;
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
// glm::rotate(m, angle, axis) = m * R(axis, angle) (glm/gtc/matrix_transform.inl)
void rot_axis(double m[3][3], int axis, double deg) {
    double a = deg * 3.14159265358979323846 / 180.0;
    double c = std::cos(a), s = std::sin(a);
    double r[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    int i = (axis + 1) % 3, j = (axis + 2) % 3;
    r[i][i] = c; r[i][j] = -s; r[j][i] = s; r[j][j] = c;
    double o[3][3];
    for (int p = 0; p < 3; p++)
        for (int q = 0; q < 3; q++) o[p][q] = m[p][0] * r[0][q] + m[p][1] * r[1][q] + m[p][2] * r[2][q];
    std::memcpy(m, o, sizeof(o));
}
inline pt_float3 norm3(double x, double y, double z) {
    float fx = (float)x, fy = (float)y, fz = (float)z;
    float inv = 1.0f / std::sqrt(fx * fx + fy * fy + fz * fz);
    return {fx * inv, fy * inv, fz * inv};
}
}  // namespace

// triangle_mesh::load_obj (:136-171, rotation) + create_mesh_device_data (:593-647, translate*scale)
extern "C" int pt_scene_builder_add_mesh(pt_scene_builder* b, int tri_num, const float* v, const float* nrm,
                                         const float* uv, const int* tri_material, pt_float3 pos, pt_float3 scl,
                                         pt_float3 rot) {
    if (!b || tri_num <= 0 || !v || !nrm || !tri_material) return -1;
    double R[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    rot_axis(R, 2, rot.z);
    rot_axis(R, 1, rot.y);
    rot_axis(R, 0, rot.x);
    const bool identity = rot.x == 0.0f && rot.y == 0.0f && rot.z == 0.0f;
    b->mesh_start.push_back((int)b->triangles.size());
    b->mesh_count.push_back(tri_num);
    for (int t = 0; t < tri_num; t++) {
        pt_triangle tr;
        std::memset(&tr, 0, sizeof(tr));
        pt_float3* vo[3] = {&tr.vertex0, &tr.vertex1, &tr.vertex2};
        pt_float3* no[3] = {&tr.normal0, &tr.normal1, &tr.normal2};
        pt_float2* uo[3] = {&tr.uv0, &tr.uv1, &tr.uv2};
        for (int k = 0; k < 3; k++) {
            const float* p = v + (size_t)t * 9 + k * 3;
            const float* q = nrm + (size_t)t * 9 + k * 3;
            float rx, ry, rz;
            double nx, ny, nz;
            if (identity) {
                rx = p[0]; ry = p[1]; rz = p[2];
                nx = q[0]; ny = q[1]; nz = q[2];
            } else {
                rx = (float)(R[0][0] * p[0] + R[0][1] * p[1] + R[0][2] * p[2]);
                ry = (float)(R[1][0] * p[0] + R[1][1] * p[1] + R[1][2] * p[2]);
                rz = (float)(R[2][0] * p[0] + R[2][1] * p[1] + R[2][2] * p[2]);
                nx = R[0][0] * q[0] + R[0][1] * q[1] + R[0][2] * q[2];
                ny = R[1][0] * q[0] + R[1][1] * q[1] + R[1][2] * q[2];
                nz = R[2][0] * q[0] + R[2][1] * q[1] + R[2][2] * q[2];
            }
            pt_float3 nr = norm3(nx, ny, nz);  // normalize after rotation (:163-165)
            *vo[k] = {scl.x * rx + pos.x, scl.y * ry + pos.y, scl.z * rz + pos.z};
            // inverse transpose of translate*scale on a direction = diag(1/s) (:633-644)
            *no[k] = norm3((double)(nr.x / scl.x), (double)(nr.y / scl.y), (double)(nr.z / scl.z));
            if (uv) *uo[k] = {uv[(size_t)t * 6 + k * 2], uv[(size_t)t * 6 + k * 2 + 1]};
            else *uo[k] = {0.0f, 0.0f};
        }
        b->triangles.push_back(tr);
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
    if (!b) return -1;
    b->release_bvh();
    for (size_t t = 0; t < b->triangles.size(); t++) {
        int m = b->tri_material[t];
        if (m < 0 || m >= (int)b->materials.size()) return -3;
        b->triangles[t].mat = b->materials.data() + m;
    }
    for (size_t m = 0; m < b->mesh_start.size(); m++) {
        pt_bvh_node_device* nodes = nullptr;
        int nn = 0, *leaf = nullptr, ln = 0;
        int rc = pt_bvh_build(b->triangles.data() + b->mesh_start[m], b->mesh_count[m], b->mesh_start[m], leaf_size,
                              method, &nodes, &nn, &leaf, &ln);
        if (rc != 0) return rc;
        b->bvh_nodes.push_back(nodes);
        b->bvh_leaf.push_back(leaf);
        b->node_num.push_back(nn);
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
