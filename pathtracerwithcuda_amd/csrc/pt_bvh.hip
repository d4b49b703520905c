// pt_bvh.hip — the MortonCodeCUDA BVH builder on gfx950 (include/pt_bvh.h).
//
// The reference builds each mesh's BVH with two CUDA kernels and two thrust::sort calls
// (Bvh/bvh.cpp:862-972, Kernel/bvh_morton_code_kernel.cu, Kernel/parallel_function.cu:22-32) and
// finishes on the host (bottom-up boxes, flattening). Here:
//   triangle_nodes_kernel   per-triangle box + 30-bit Morton code of its centroid in the mesh box
//   radix sort              hipcub stable LSD radix sort of (code, index) over 30 bits, then a gather
//                           of the 64-B node records (thrust's comparator sort is a stable merge sort)
//   batch_leaves_kernel     leaf_size consecutive sorted triangles per leaf, leaf box, leaf code
//                           (the reference batches on the host, bvh.cpp:920-955)
//   internal_nodes_kernel   Karras split/range per internal node; parent links resolved with
//                           atomicMax so the largest writer wins (the reference races here)
// then the second half — bottom-up boxes and the preorder flatten — on the device too (fin_* kernels)
// for a well-formed tree, or the host builder's own second half (pt_morton_finish) otherwise; either
// way the two builders' node arrays are identical.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/pt_bvh.h"
#include "pt_bvh_common.h"
#include "pt_bvh_internal.h"

namespace {

constexpr int kBlock = 256;

#define BVH_HIP(call)                                                                                      \
    do {                                                                                                   \
        hipError_t e_ = (call);                                                                            \
        if (e_ != hipSuccess) {                                                                            \
            std::fprintf(stderr, "[Hip]Error %s in file %s line %d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return e_;                                                                                     \
        }                                                                                                  \
    } while (0)

__device__ __forceinline__ ptbvh::Box to_box(const pt_bounding_box& b) {
    ptbvh::Box r;
    r.lb[0] = b.left_bottom.x; r.lb[1] = b.left_bottom.y; r.lb[2] = b.left_bottom.z;
    r.rt[0] = b.right_top.x; r.rt[1] = b.right_top.y; r.rt[2] = b.right_top.z;
    return r;
}

__device__ __forceinline__ void store_box(pt_bounding_box& d, const ptbvh::Box& b) {  // get_bounding_box
    d.left_bottom = {b.lb[0], b.lb[1], b.lb[2]};
    d.right_top = {b.rt[0], b.rt[1], b.rt[2]};
    d.centroid = {0.5f * (b.rt[0] + b.lb[0]), 0.5f * (b.rt[1] + b.lb[1]), 0.5f * (b.rt[2] + b.lb[2])};
}

// __compute_triangle_bounding_box_kernel (bvh_morton_code_kernel.cu:298-326)
__global__ __launch_bounds__(kBlock) void triangle_nodes_kernel(const pt_triangle* __restrict__ tris, int n,
                                                                pt_bvh_node_morton_code_cuda* __restrict__ out,
                                                                const pt_bounding_box* __restrict__ mesh_box,
                                                                int start_index) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const pt_triangle& t = tris[i];
    const ptbvh::Box b = ptbvh::box_of_vertices(&t.vertex0.x, &t.vertex1.x, &t.vertex2.x);
    pt_bvh_node_morton_code_cuda& o = out[i];
    o.triangle_index = i + start_index;
    store_box(o.box, b);
    o.morton_code = ptbvh::morton_of_box(b, to_box(*mesh_box));
}

__global__ __launch_bounds__(kBlock) void sort_keys_kernel(const pt_bvh_node_morton_code_cuda* __restrict__ in, int n,
                                                           unsigned int* __restrict__ keys, int* __restrict__ idx) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    keys[i] = in[i].morton_code;
    idx[i] = i;
}

__global__ __launch_bounds__(kBlock) void gather_kernel(const pt_bvh_node_morton_code_cuda* __restrict__ in, int n,
                                                        const int* __restrict__ idx,
                                                        pt_bvh_node_morton_code_cuda* __restrict__ out) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    out[i] = in[idx[i]];
}

// bvh.cpp:924-956 (host loop in the reference): triangle_index = batch id, slots -1 padded
__global__ __launch_bounds__(kBlock) void batch_leaves_kernel(const pt_bvh_node_morton_code_cuda* __restrict__ tri_sorted,
                                                              int n, int leaf_size, unsigned int leaf_num,
                                                              pt_bvh_node_morton_code_cuda* __restrict__ leaves,
                                                              int* __restrict__ batch_tris,
                                                              const pt_bounding_box* __restrict__ mesh_box) {
    const unsigned int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= leaf_num) return;
    const int s = (int)i * leaf_size;
    ptbvh::Box b = to_box(tri_sorted[s].box);
    batch_tris[(size_t)i * leaf_size] = tri_sorted[s].triangle_index;
    for (int j = 1; j < leaf_size; j++) {
        int tri = -1;
        if (j + s < n) {
            ptbvh::expand(b, to_box(tri_sorted[j + s].box));
            tri = tri_sorted[j + s].triangle_index;
        }
        batch_tris[(size_t)i * leaf_size + j] = tri;
    }
    pt_bvh_node_morton_code_cuda o;
    store_box(o.box, b);
    o.left_index = -1; o.right_index = -1; o.parent_index = -1;
    o.is_left_leaf = 0; o.is_right_leaf = 0; o.is_leaf = 1;
    o.triangle_index = (int)i;
    o.morton_code = ptbvh::morton_of_box(b, to_box(*mesh_box));
    o.is_visited = -1;
    leaves[i] = o;
}

__global__ __launch_bounds__(kBlock) void reset_parents_kernel(pt_bvh_node_morton_code_cuda* __restrict__ nodes,
                                                               unsigned int count) {
    const unsigned int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < count) nodes[i].parent_index = -1;
}

// ---- the second half on the device (bottom-up boxes, preorder flatten) ------------------------------
// The reference finishes each mesh on the host: every leaf walks to the root unioning boxes (bvh.cpp:
// 817-860, 974-982), then a stack-based preorder flatten assigns skip indices (:244-330). For a
// well-formed Karras tree (every node but the root referenced by exactly one internal node — checked
// by fin_refs/fin_check; otherwise the host finish runs) the same arrays come out of four kernels:
//   fin_refs      child -> parent links and reference counts (keys: internal i, leaf I + l)
//   fin_up        one thread per leaf climbs with an arrival counter per internal node: the second
//                 child to arrive unions the two boxes (left first, as the host fold) and the subtree
//                 sizes, then climbs on; agent-scope release/acquire around the counter
//   fin_flatten   each node's preorder position from its path to the root (+1 per ancestor, + the left
//                 sibling's subtree size when it is a right child); next = position + subtree size;
//                 a thin leaf box is widened by its parent's box (bvh.cpp:265-268); node records and
//                 the leaf triangle slots written in place (leaves keep the sorted order in preorder)
struct FinTree {
    const pt_bvh_node_morton_code_cuda* inner;   // I internal nodes (children, leaf flags)
    const pt_bvh_node_morton_code_cuda* leaves;  // L sorted leaves (box, batch id)
    const int* batch_tris;                       // L * leaf_size triangle ids by batch
    int* parent;                                 // I + L: the referring internal node
    int* is_right;                               // I + L: 1 when the node is its parent's right child
    int* refs;                                   // I + L
    unsigned int* arrive;                        // I
    float* inner_box;                            // I * 6
    int* size;                                   // I + L subtree sizes (leaves 1)
    int* bad;                                    // set when the tree is not well formed
    unsigned int I, L;
};

__device__ __forceinline__ int fin_child_key(const FinTree& t, int index, int is_leaf) {
    return is_leaf ? (int)t.I + index : index;
}

__global__ __launch_bounds__(kBlock) void fin_refs_kernel(FinTree t) {
    const unsigned int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= t.I) return;
    const pt_bvh_node_morton_code_cuda& n = t.inner[i];
    const int l = fin_child_key(t, n.left_index, n.is_left_leaf), r = fin_child_key(t, n.right_index, n.is_right_leaf);
    const int total = (int)(t.I + t.L);
    if (l < 0 || l >= total || r < 0 || r >= total || l == r) { atomicOr(t.bad, 1); return; }
    atomicAdd(&t.refs[l], 1);
    atomicAdd(&t.refs[r], 1);
    t.parent[l] = (int)i; t.is_right[l] = 0;
    t.parent[r] = (int)i; t.is_right[r] = 1;
}

__global__ __launch_bounds__(kBlock) void fin_check_kernel(FinTree t) {
    const unsigned int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= t.I + t.L) return;
    if (t.refs[k] != (k == 0 ? 0 : 1)) atomicOr(t.bad, 1);
}

__device__ __forceinline__ ptbvh::Box fin_box(const FinTree& t, int key) {
    if (key >= (int)t.I) return to_box(t.leaves[key - (int)t.I].box);
    const float* b = t.inner_box + (size_t)key * 6;
    ptbvh::Box r;
    r.lb[0] = b[0]; r.lb[1] = b[1]; r.lb[2] = b[2]; r.rt[0] = b[3]; r.rt[1] = b[4]; r.rt[2] = b[5];
    return r;
}

__global__ __launch_bounds__(kBlock) void fin_up_kernel(FinTree t) {
    const unsigned int l = blockIdx.x * kBlock + threadIdx.x;
    if (l >= t.L) return;
    int key = (int)(t.I + l);
    t.size[key] = 1;
    while (key != 0) {
        const int p = t.parent[key];
        // publish this subtree's box and size, then arrive; the second arrival finishes the parent
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned int old = atomicAdd(&t.arrive[p], 1u);
        if (old == 0) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const pt_bvh_node_morton_code_cuda& n = t.inner[p];
        const int lk = fin_child_key(t, n.left_index, n.is_left_leaf), rk = fin_child_key(t, n.right_index, n.is_right_leaf);
        ptbvh::Box b = fin_box(t, lk);  // bvh.cpp:837-848: the left child's box expanded by the right's
        ptbvh::expand(b, fin_box(t, rk));
        float* o = t.inner_box + (size_t)p * 6;
        o[0] = b.lb[0]; o[1] = b.lb[1]; o[2] = b.lb[2]; o[3] = b.rt[0]; o[4] = b.rt[1]; o[5] = b.rt[2];
        t.size[p] = 1 + t.size[lk] + t.size[rk];
        key = p;
    }
}

// pt_bvh_node_device (include/pt_types.h) as the kernel writes it: the leaf slot pointer is the host
// address the finished array will have
__global__ __launch_bounds__(kBlock) void fin_flatten_kernel(FinTree t, pt_bvh_node_device* __restrict__ out,
                                                             int* __restrict__ leaf_slots, int leaf_size,
                                                             unsigned long long host_leaf_base) {
    const unsigned int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= t.I + t.L) return;
    // preorder position: one per ancestor, plus the left sibling's subtree whenever the path turns right.
    // The climb is capped at I + L links: a node on (or below) a cycle never reaches the root, which the
    // host's size[0] check before this launch rules out; the cap keeps a missed case from hanging the GPU.
    int pos = 0;
    unsigned int hops = 0;
    for (int c = (int)k; c != 0;) {
        if (++hops > t.I + t.L) { atomicOr(t.bad, 1); return; }
        const int p = t.parent[c];
        pos += 1;
        if (t.is_right[c]) {
            const pt_bvh_node_morton_code_cuda& n = t.inner[p];
            pos += t.size[fin_child_key(t, n.left_index, n.is_left_leaf)];
        }
        c = p;
    }
    const bool leaf = k >= t.I;
    ptbvh::Box b = fin_box(t, (int)k);
    if (leaf && ptbvh::is_thin(b)) ptbvh::expand(b, fin_box(t, t.parent[k]));
    pt_bvh_node_device& d = out[pos];
    store_box(d.box, b);
    d.is_leaf = leaf ? 1 : 0;
    d.next_node_index = pos + t.size[k];
    if (leaf) {
        const unsigned int l = k - t.I;
        const int batch = t.leaves[l].triangle_index;
        for (int j = 0; j < leaf_size; j++)
            leaf_slots[(size_t)l * leaf_size + j] = t.batch_tris[(size_t)batch * leaf_size + j];
        d.triangle_indices = (int*)(host_leaf_base + (unsigned long long)l * leaf_size * sizeof(int));
    } else {
        d.triangle_indices = nullptr;
    }
}

struct LeafCodes {
    const pt_bvh_node_morton_code_cuda* leaves;
    __device__ unsigned int operator[](unsigned int k) const { return leaves[k].morton_code; }
};

// __generate_internal_node_kernel + generate_internal_node (bvh_morton_code_kernel.cu:250-346)
__global__ __launch_bounds__(kBlock) void internal_nodes_kernel(pt_bvh_node_morton_code_cuda* __restrict__ internal,
                                                                unsigned int internal_num,
                                                                pt_bvh_node_morton_code_cuda* __restrict__ leaves,
                                                                unsigned int leaf_num) {
    const unsigned int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= internal_num) return;
    const LeafCodes codes{leaves};
    unsigned int rx, ry;
    ptbvh::find_range(codes, leaf_num, i, &rx, &ry);
    const unsigned int split = ptbvh::find_split(codes, rx, ry);
    const bool left_leaf = split == rx, right_leaf = split + 1 == ry;
    atomicMax(left_leaf ? &leaves[split].parent_index : &internal[split].parent_index, (int)i);
    atomicMax(right_leaf ? &leaves[split + 1].parent_index : &internal[split + 1].parent_index, (int)i);
    internal[i].left_index = (int)split;
    internal[i].right_index = (int)split + 1;
    internal[i].is_left_leaf = left_leaf ? 1 : 0;
    internal[i].is_right_leaf = right_leaf ? 1 : 0;
}

inline unsigned int grid_of(size_t n) { return (unsigned int)((n + kBlock - 1) / kBlock); }

// Stable sort of node records by morton_code (device in, device out).
hipError_t sort_nodes(const pt_bvh_node_morton_code_cuda* in, pt_bvh_node_morton_code_cuda* out, int n,
                      hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    unsigned int *k0 = nullptr, *k1 = nullptr;
    int *v0 = nullptr, *v1 = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    hipError_t e = hipMalloc(&k0, sizeof(unsigned int) * n);
    if (e == hipSuccess) e = hipMalloc(&k1, sizeof(unsigned int) * n);
    if (e == hipSuccess) e = hipMalloc(&v0, sizeof(int) * n);
    if (e == hipSuccess) e = hipMalloc(&v1, sizeof(int) * n);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(sort_keys_kernel, dim3(grid_of(n)), dim3(kBlock), 0, stream, in, n, k0, v0);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k0, k1, v0, v1, n, 0, 30, stream);
    if (e == hipSuccess) e = hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 1);
    if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, v0, v1, n, 0, 30, stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(gather_kernel, dim3(grid_of(n)), dim3(kBlock), 0, stream, in, n, v1, out);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    (void)hipFree(k0); (void)hipFree(k1); (void)hipFree(v0); (void)hipFree(v1); (void)hipFree(tmp);
    return e;
}

bool is_device_memory(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.type == hipMemoryTypeUnified;
}

// A caller buffer as device memory: used in place when it already is, else staged through HBM
// (copied in on construction when `in`, copied back by finish() when `out`).
template <class T>
struct Staged {
    T* user = nullptr;
    T* dev = nullptr;
    size_t count = 0;
    bool owned = false;
    hipError_t init(T* p, size_t n, bool in) {
        user = p; count = n;
        if (!p || n == 0 || is_device_memory(p)) { dev = p; return hipSuccess; }
        owned = true;
        hipError_t e = hipMalloc(&dev, sizeof(T) * n);
        if (e == hipSuccess && in) e = hipMemcpy(dev, p, sizeof(T) * n, hipMemcpyHostToDevice);
        return e;
    }
    hipError_t finish(bool out) {
        hipError_t e = hipSuccess;
        if (owned && out) e = hipMemcpy(user, dev, sizeof(T) * count, hipMemcpyDeviceToHost);
        if (owned) (void)hipFree(dev);
        owned = false;
        return e;
    }
    ~Staged() { if (owned) (void)hipFree(dev); }
};

void report(hipError_t e, const char* what) {
    if (e != hipSuccess) std::fprintf(stderr, "[Hip]Error %s in %s\n", hipGetErrorString(e), what);
}

}  // namespace

extern "C" void compute_triangle_bounding_box_kernel(pt_triangle* triangles, int triangle_num,
                                                     pt_bvh_node_morton_code_cuda* triangle_nodes,
                                                     pt_bounding_box* mesh_box, int start_index, int block_size) {
    (void)block_size;
    if (triangle_num <= 0 || !triangles || !triangle_nodes || !mesh_box) return;
    Staged<pt_triangle> t;
    Staged<pt_bvh_node_morton_code_cuda> o;
    Staged<pt_bounding_box> m;
    hipError_t e = t.init(triangles, (size_t)triangle_num, true);
    if (e == hipSuccess) e = o.init(triangle_nodes, (size_t)triangle_num, true);
    if (e == hipSuccess) e = m.init(mesh_box, 1, true);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(triangle_nodes_kernel, dim3(grid_of((size_t)triangle_num)), dim3(kBlock), 0, 0, t.dev,
                           triangle_num, o.dev, m.dev, start_index);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = o.finish(true);
    report(e, "compute_triangle_bounding_box_kernel");
}

extern "C" void generate_internal_node_kernel(pt_bvh_node_morton_code_cuda* internal_nodes, unsigned int internal_node_num,
                                              pt_bvh_node_morton_code_cuda* leaf_nodes, unsigned int leaf_node_num,
                                              int block_size) {
    (void)block_size;
    if (internal_node_num == 0 || !internal_nodes || !leaf_nodes || leaf_node_num != internal_node_num + 1) return;
    Staged<pt_bvh_node_morton_code_cuda> in, lf;
    hipError_t e = in.init(internal_nodes, internal_node_num, true);
    if (e == hipSuccess) e = lf.init(leaf_nodes, leaf_node_num, true);
    if (e == hipSuccess) {
        // the reference leaves parent links of non-root nodes to whichever parent writes last; here the
        // links are reset, then resolved deterministically (largest parent index)
        hipLaunchKernelGGL(reset_parents_kernel, dim3(grid_of(internal_node_num)), dim3(kBlock), 0, 0, in.dev,
                           internal_node_num);
        hipLaunchKernelGGL(reset_parents_kernel, dim3(grid_of(leaf_node_num)), dim3(kBlock), 0, 0, lf.dev, leaf_node_num);
        hipLaunchKernelGGL(internal_nodes_kernel, dim3(grid_of(internal_node_num)), dim3(kBlock), 0, 0, in.dev,
                           internal_node_num, lf.dev, leaf_node_num);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = in.finish(true);
    if (e == hipSuccess) e = lf.finish(true);
    report(e, "generate_internal_node_kernel");
}

extern "C" void radix_sort(pt_bvh_node_morton_code_cuda* arrays, pt_bvh_node_morton_code_cuda* sorted_arrays, int number) {
    if (number <= 0 || !arrays || !sorted_arrays) return;
    Staged<pt_bvh_node_morton_code_cuda> in, out;
    hipError_t e = in.init(arrays, (size_t)number, true);
    if (e == hipSuccess) e = out.init(sorted_arrays, (size_t)number, false);
    if (e == hipSuccess) e = sort_nodes(in.dev, out.dev, number, 0);
    if (e == hipSuccess) e = out.finish(true);
    report(e, "radix_sort");
}

extern "C" int pt_bvh_build_device(const pt_triangle* tris, int n, int start_index, int leaf_size,
                                   pt_bvh_node_device** nodes_out, int* node_num_out, int** leaf_out, int* leaf_num_out) {
    if (!tris || n <= 0 || leaf_size <= 0 || !nodes_out || !node_num_out || !leaf_out || !leaf_num_out) return -1;
    PtMortonTree t;
    t.leaf_num = pt_leaf_count(n, leaf_size);
    t.internal_num = t.leaf_num - 1;
    const unsigned int L = t.leaf_num, I = t.internal_num;

    // the mesh box is a sequential fold on the host in the reference too (bvh.cpp:889-895)
    ptbvh::Box mesh = ptbvh::box_of_vertices(&tris[0].vertex0.x, &tris[0].vertex1.x, &tris[0].vertex2.x);
    for (int i = 1; i < n; i++)
        ptbvh::expand(mesh, ptbvh::box_of_vertices(&tris[i].vertex0.x, &tris[i].vertex1.x, &tris[i].vertex2.x));
    pt_bounding_box mesh_box;
    mesh_box.left_bottom = {mesh.lb[0], mesh.lb[1], mesh.lb[2]};
    mesh_box.right_top = {mesh.rt[0], mesh.rt[1], mesh.rt[2]};
    mesh_box.centroid = {0.5f * (mesh.rt[0] + mesh.lb[0]), 0.5f * (mesh.rt[1] + mesh.lb[1]), 0.5f * (mesh.rt[2] + mesh.lb[2])};

    hipStream_t stream = nullptr;
    pt_triangle* d_tris = nullptr;
    pt_bvh_node_morton_code_cuda *d_tn = nullptr, *d_tn_sorted = nullptr, *d_leaf = nullptr, *d_leaf_sorted = nullptr,
                                 *d_internal = nullptr;
    pt_bounding_box* d_mesh = nullptr;
    int* d_batch = nullptr;
    std::vector<pt_bvh_node_morton_code_cuda> h_leaf(L), h_internal(I);
    t.batch_tris.resize((size_t)L * leaf_size);
    // PT_BVH_DEVICE_FINISH=0: bottom-up boxes and flattening on the host (pt_morton_finish) as before
    static const bool device_finish = [] {
        const char* e = std::getenv("PT_BVH_DEVICE_FINISH");
        return !(e && std::atoi(e) == 0);
    }();
    bool finished = false;
    void* d_fin = nullptr;
    pt_bvh_node_device* h_nodes = nullptr;
    int* h_leaf_idx = nullptr;
    // the second half on the device (fin_* kernels): false `finished` = the tree is not well formed and
    // the host finish runs on the downloaded arrays
    auto finish_on_device = [&]() -> hipError_t {
        const size_t K = (size_t)I + L, N = K;
        size_t off = 0;
        auto take = [&](size_t bytes) { const size_t o = off; off = (off + bytes + 255) & ~(size_t)255; return o; };
        const size_t o_parent = take(K * 4), o_right = take(K * 4), o_refs = take(K * 4), o_arrive = take((size_t)I * 4),
                     o_box = take((size_t)I * 24), o_size = take(K * 4), o_bad = take(4),
                     o_out = take(N * sizeof(pt_bvh_node_device)), o_slots = take((size_t)L * leaf_size * 4);
        BVH_HIP(hipMalloc(&d_fin, off));
        uint8_t* base = (uint8_t*)d_fin;
        BVH_HIP(hipMemsetAsync(base, 0, off, stream));
        FinTree ft;
        ft.inner = d_internal;
        ft.leaves = d_leaf_sorted;
        ft.batch_tris = d_batch;
        ft.parent = (int*)(base + o_parent);
        ft.is_right = (int*)(base + o_right);
        ft.refs = (int*)(base + o_refs);
        ft.arrive = (unsigned int*)(base + o_arrive);
        ft.inner_box = (float*)(base + o_box);
        ft.size = (int*)(base + o_size);
        ft.bad = (int*)(base + o_bad);
        ft.I = I;
        ft.L = L;
        hipLaunchKernelGGL(fin_refs_kernel, dim3(grid_of(I)), dim3(kBlock), 0, stream, ft);
        hipLaunchKernelGGL(fin_check_kernel, dim3(grid_of((unsigned int)K)), dim3(kBlock), 0, stream, ft);
        BVH_HIP(hipGetLastError());
        int bad = 0;
        BVH_HIP(hipMemcpyAsync(&bad, ft.bad, 4, hipMemcpyDeviceToHost, stream));
        BVH_HIP(hipStreamSynchronize(stream));
        if (bad) return hipSuccess;  // host finish
        h_nodes = (pt_bvh_node_device*)std::calloc(N, sizeof(pt_bvh_node_device));
        h_leaf_idx = (int*)std::malloc((size_t)L * leaf_size * sizeof(int));
        if (!h_nodes || !h_leaf_idx) return hipErrorOutOfMemory;
        pt_bvh_node_device* d_out = (pt_bvh_node_device*)(base + o_out);
        int* d_slots = (int*)(base + o_slots);
        hipLaunchKernelGGL(fin_up_kernel, dim3(grid_of(L)), dim3(kBlock), 0, stream, ft);
        BVH_HIP(hipGetLastError());
        // fin_refs/fin_check count references only: a component holding a cycle (a -> b -> a, each with one
        // other child) passes them, and its nodes never reach the root. The root's subtree then holds fewer
        // than I + L nodes: such a tree takes the host finish (its explicit stack visits each node once).
        int root_size = 0;
        BVH_HIP(hipMemcpyAsync(&root_size, ft.size, 4, hipMemcpyDeviceToHost, stream));
        BVH_HIP(hipStreamSynchronize(stream));
        if (root_size != (int)K) return hipSuccess;  // host finish
        hipLaunchKernelGGL(fin_flatten_kernel, dim3(grid_of((unsigned int)K)), dim3(kBlock), 0, stream, ft, d_out, d_slots,
                           leaf_size, (unsigned long long)(uintptr_t)h_leaf_idx);
        BVH_HIP(hipGetLastError());
        BVH_HIP(hipMemcpyAsync(h_nodes, d_out, N * sizeof(pt_bvh_node_device), hipMemcpyDeviceToHost, stream));
        BVH_HIP(hipMemcpyAsync(h_leaf_idx, d_slots, (size_t)L * leaf_size * sizeof(int), hipMemcpyDeviceToHost, stream));
        BVH_HIP(hipMemcpyAsync(&bad, ft.bad, 4, hipMemcpyDeviceToHost, stream));
        BVH_HIP(hipStreamSynchronize(stream));
        if (bad) return hipSuccess;  // host finish
        finished = true;
        return hipSuccess;
    };
    auto run = [&]() -> hipError_t {
        BVH_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        BVH_HIP(hipMalloc(&d_tris, sizeof(pt_triangle) * n));
        BVH_HIP(hipMalloc(&d_tn, sizeof(pt_bvh_node_morton_code_cuda) * n));
        BVH_HIP(hipMalloc(&d_tn_sorted, sizeof(pt_bvh_node_morton_code_cuda) * n));
        BVH_HIP(hipMalloc(&d_leaf, sizeof(pt_bvh_node_morton_code_cuda) * L));
        BVH_HIP(hipMalloc(&d_leaf_sorted, sizeof(pt_bvh_node_morton_code_cuda) * L));
        BVH_HIP(hipMalloc(&d_internal, sizeof(pt_bvh_node_morton_code_cuda) * (I ? I : 1)));
        BVH_HIP(hipMalloc(&d_mesh, sizeof(pt_bounding_box)));
        BVH_HIP(hipMalloc(&d_batch, sizeof(int) * L * leaf_size));
        BVH_HIP(hipMemcpyAsync(d_tris, tris, sizeof(pt_triangle) * n, hipMemcpyHostToDevice, stream));
        BVH_HIP(hipMemcpyAsync(d_mesh, &mesh_box, sizeof(mesh_box), hipMemcpyHostToDevice, stream));
        hipLaunchKernelGGL(triangle_nodes_kernel, dim3(grid_of(n)), dim3(kBlock), 0, stream, d_tris, n, d_tn, d_mesh,
                           start_index);
        BVH_HIP(hipGetLastError());
        BVH_HIP(sort_nodes(d_tn, d_tn_sorted, n, stream));
        hipLaunchKernelGGL(batch_leaves_kernel, dim3(grid_of(L)), dim3(kBlock), 0, stream, d_tn_sorted, n, leaf_size, L,
                           d_leaf, d_batch, d_mesh);
        BVH_HIP(hipGetLastError());
        BVH_HIP(sort_nodes(d_leaf, d_leaf_sorted, (int)L, stream));
        if (I > 0) {
            hipLaunchKernelGGL(reset_parents_kernel, dim3(grid_of(I)), dim3(kBlock), 0, stream, d_internal, I);
            hipLaunchKernelGGL(internal_nodes_kernel, dim3(grid_of(I)), dim3(kBlock), 0, stream, d_internal, I,
                               d_leaf_sorted, L);
            BVH_HIP(hipGetLastError());
            if (device_finish) {
                BVH_HIP(finish_on_device());
                if (finished) return hipSuccess;
            }
            BVH_HIP(hipMemcpyAsync(h_internal.data(), d_internal, sizeof(pt_bvh_node_morton_code_cuda) * I,
                                   hipMemcpyDeviceToHost, stream));
        }
        BVH_HIP(hipMemcpyAsync(h_leaf.data(), d_leaf_sorted, sizeof(pt_bvh_node_morton_code_cuda) * L,
                               hipMemcpyDeviceToHost, stream));
        BVH_HIP(hipMemcpyAsync(t.batch_tris.data(), d_batch, sizeof(int) * L * leaf_size, hipMemcpyDeviceToHost, stream));
        BVH_HIP(hipStreamSynchronize(stream));
        return hipSuccess;
    };
    const hipError_t e = run();
    if (d_fin) (void)hipFree(d_fin);
    (void)hipFree(d_tris); (void)hipFree(d_tn); (void)hipFree(d_tn_sorted); (void)hipFree(d_leaf);
    (void)hipFree(d_leaf_sorted); (void)hipFree(d_internal); (void)hipFree(d_mesh); (void)hipFree(d_batch);
    if (stream) (void)hipStreamDestroy(stream);
    if (e != hipSuccess || !finished) {
        std::free(h_nodes);
        std::free(h_leaf_idx);
        if (e != hipSuccess) return -3;
    } else {
        *nodes_out = h_nodes;
        *node_num_out = (int)(L + I);
        *leaf_out = h_leaf_idx;
        *leaf_num_out = (int)L;
        return 0;
    }

    t.leaf_box.resize(L);
    t.leaf_batch.resize(L);
    t.leaf_parent.resize(L);
    for (unsigned int i = 0; i < L; i++) {
        const pt_bounding_box& b = h_leaf[i].box;
        t.leaf_box[i] = ptbvh::Box{{b.left_bottom.x, b.left_bottom.y, b.left_bottom.z}, {b.right_top.x, b.right_top.y, b.right_top.z}};
        t.leaf_batch[i] = h_leaf[i].triangle_index;
        t.leaf_parent[i] = h_leaf[i].parent_index;
    }
    t.inner_left.resize(I);
    t.inner_right.resize(I);
    t.inner_parent.resize(I);
    for (unsigned int i = 0; i < I; i++) {
        const pt_bvh_node_morton_code_cuda& x = h_internal[i];
        t.inner_left[i] = x.is_left_leaf ? -(x.left_index + 2) : x.left_index;
        t.inner_right[i] = x.is_right_leaf ? -(x.right_index + 2) : x.right_index;
        t.inner_parent[i] = i == 0 ? -1 : x.parent_index;
    }
    return pt_morton_finish(t, leaf_size, nodes_out, node_num_out, leaf_out, leaf_num_out);
}
