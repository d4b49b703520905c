// pt_bvh_sah.hip — PT_BVH_SAH on gfx950: the binned true-surface-area tree of pt_host.cpp (pt_bvh_build_sah), built
// on the device, node for node the same tree (include/pt_host.h).
//
// The host builder splits one node at a time (explicit stack). Here the tree grows level by level: one launch of
// sah_level_kernel per level, one workgroup per node of the level, which
//   1. reduces the node's box and centroid bounds over its triangles (its range of the index array),
//   2. makes a leaf (<= leaf_size triangles) or bins the centroids per axis in LDS (counts, boxes by ordered-int
//      atomics: min/max are order-independent),
//   3. sweeps the bins exactly as the host does (same float bin arithmetic, surface areas in double, the first
//      strictly smaller cost in axis-then-bin order),
//   4. partitions its range stably (ballot scans over 256-triangle chunks, as std::stable_partition orders them) and
//      appends its two children, in the host's child order, to the next level.
// Node numbers differ from the host's (atomic allocation); the tree does not, and the flattening (preorder, skip
// indices, thin leaf boxes widened, pt_flatten_tree) runs on the host over the downloaded tree, so both builders
// give the same node array byte for byte (tests/test_bvh_device.py).
//
// Signed zeros: both builders take the triangle boxes with -0 turned into +0 (ptbvh::canonical_zeros), since the
// host's a < b ? a : b union keeps whichever zero came last; a zero's sign changes no slab-test outcome.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/pt_host.h"
#include "pt_bvh_common.h"
#include "pt_bvh_internal.h"

namespace {

constexpr int kSahBlock = 256;
constexpr int kMaxBins = 64;

#define SAH_HIP(call)                                                                                      \
    do {                                                                                                   \
        hipError_t e_ = (call);                                                                            \
        if (e_ != hipSuccess) {                                                                            \
            std::fprintf(stderr, "[Hip]Error %s in file %s line %d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return e_;                                                                                     \
        }                                                                                                  \
    } while (0)

struct SahTask {
    int node, begin, end;
};

struct SahTree {
    float* box;    // 6 floats per node: lb xyz, rt xyz
    int* left;     // child node ids (-1: leaf)
    int* right;
    int* begin;    // a leaf's range of idx
    int* end;
    int* count;    // [0] nodes allocated, [1] tasks of the next level
};

// float <-> an int whose signed order is the float order (for LDS atomicMin / atomicMax)
__device__ __forceinline__ int ord(float f) {
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float unord(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

__device__ __forceinline__ double sa_of(const float* lb, const float* rt) {
    const double x = (double)rt[0] - lb[0], y = (double)rt[1] - lb[1], z = (double)rt[2] - lb[2];
    return 2.0 * (x * y + y * z + z * x);
}

__global__ __launch_bounds__(kSahBlock) void sah_prepare_kernel(const pt_triangle* __restrict__ tris, int n,
                                                                float* __restrict__ tbox, float* __restrict__ cen,
                                                                int* __restrict__ idx) {
    const int i = blockIdx.x * kSahBlock + threadIdx.x;
    if (i >= n) return;
    const pt_triangle& t = tris[i];
    ptbvh::Box b = ptbvh::box_of_vertices(&t.vertex0.x, &t.vertex1.x, &t.vertex2.x);
    ptbvh::canonical_zeros(b);
    for (int k = 0; k < 3; k++) {
        tbox[(size_t)i * 6 + k] = b.lb[k];
        tbox[(size_t)i * 6 + 3 + k] = b.rt[k];
        cen[(size_t)i * 3 + k] = 0.5f * (b.lb[k] + b.rt[k]);
    }
    idx[i] = i;
}

// block-wide min (is_max false) / max of one float per thread, by ordered ints in LDS
__device__ __forceinline__ float block_extreme(float v, bool is_max, int* slot) {
    if (threadIdx.x == 0) *slot = is_max ? INT_MIN : INT_MAX;
    __syncthreads();
    if (is_max) atomicMax(slot, ord(v));
    else atomicMin(slot, ord(v));
    __syncthreads();
    const float r = unord(*slot);
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(kSahBlock) void sah_level_kernel(const float* __restrict__ tbox, const float* __restrict__ cen,
                                                              int* __restrict__ idx, int* __restrict__ tmp,
                                                              const SahTask* __restrict__ tasks, SahTask* __restrict__ next,
                                                              SahTree tree, int leaf_size, int bins, int order) {
    const SahTask task = tasks[blockIdx.x];
    const int b = task.begin, e = task.end, cnt = e - b;
    __shared__ int s_slot;
    __shared__ int s_bcnt[3][kMaxBins];
    __shared__ int s_bbox[3][kMaxBins][6];
    __shared__ int s_wave[kSahBlock / 64 + 1];
    __shared__ int s_split[4];      // axis, bin, left count, first child swap
    __shared__ float s_child[2][6]; // the two children's boxes (order 1)

    // 1. the node's box and centroid bounds
    float lo[3], hi[3], clo[3], chi[3];
    for (int k = 0; k < 3; k++) { lo[k] = clo[k] = INFINITY; hi[k] = chi[k] = -INFINITY; }
    for (int i = b + threadIdx.x; i < e; i += kSahBlock) {
        const int j = idx[i];
        for (int k = 0; k < 3; k++) {
            lo[k] = fminf(lo[k], tbox[(size_t)j * 6 + k]);
            hi[k] = fmaxf(hi[k], tbox[(size_t)j * 6 + 3 + k]);
            clo[k] = fminf(clo[k], cen[(size_t)j * 3 + k]);
            chi[k] = fmaxf(chi[k], cen[(size_t)j * 3 + k]);
        }
    }
    for (int k = 0; k < 3; k++) {
        lo[k] = block_extreme(lo[k], false, &s_slot);
        hi[k] = block_extreme(hi[k], true, &s_slot);
        clo[k] = block_extreme(clo[k], false, &s_slot);
        chi[k] = block_extreme(chi[k], true, &s_slot);
    }
    if (threadIdx.x == 0) {
        for (int k = 0; k < 3; k++) {
            tree.box[(size_t)task.node * 6 + k] = lo[k];
            tree.box[(size_t)task.node * 6 + 3 + k] = hi[k];
        }
    }
    if (cnt <= leaf_size) {  // a leaf: its triangles are idx[b, e)
        if (threadIdx.x == 0) {
            tree.left[task.node] = tree.right[task.node] = -1;
            tree.begin[task.node] = b;
            tree.end[task.node] = e;
        }
        return;
    }

    // 2. bins: counts and boxes per axis
    for (int i = threadIdx.x; i < 3 * bins; i += kSahBlock) {
        const int k = i / bins, c = i % bins;
        s_bcnt[k][c] = 0;
        for (int q = 0; q < 3; q++) { s_bbox[k][c][q] = INT_MAX; s_bbox[k][c][3 + q] = INT_MIN; }
    }
    __syncthreads();
    float scale[3];
    for (int k = 0; k < 3; k++) {
        const float ext = chi[k] - clo[k];
        scale[k] = ext > 0.0f ? (float)bins / ext : 0.0f;
    }
    for (int i = b + threadIdx.x; i < e; i += kSahBlock) {
        const int j = idx[i];
        for (int k = 0; k < 3; k++) {
            if (!(chi[k] - clo[k] > 0.0f)) continue;
            const int c = min(bins - 1, (int)((cen[(size_t)j * 3 + k] - clo[k]) * scale[k]));
            atomicAdd(&s_bcnt[k][c], 1);
            for (int q = 0; q < 3; q++) {
                atomicMin(&s_bbox[k][c][q], ord(tbox[(size_t)j * 6 + q]));
                atomicMax(&s_bbox[k][c][3 + q], ord(tbox[(size_t)j * 6 + 3 + q]));
            }
        }
    }
    __syncthreads();

    // 3. the host's sweep (pt_host.cpp sah_build), one thread
    if (threadIdx.x == 0) {
        double best = INFINITY;
        int best_axis = -1, best_bin = 0, best_nl = 0;
        double right_sa[kMaxBins];
        int right_n[kMaxBins];
        for (int k = 0; k < 3; k++) {
            if (!(chi[k] - clo[k] > 0.0f)) continue;
            float alb[3], art[3];
            bool any = false;
            int nr = 0;
            for (int c = bins - 1; c >= 1; c--) {
                if (s_bcnt[k][c]) {
                    for (int q = 0; q < 3; q++) {
                        const float l = unord(s_bbox[k][c][q]), r = unord(s_bbox[k][c][3 + q]);
                        alb[q] = any ? (alb[q] < l ? alb[q] : l) : l;
                        art[q] = any ? (art[q] > r ? art[q] : r) : r;
                    }
                    any = true;
                }
                nr += s_bcnt[k][c];
                right_sa[c] = any ? sa_of(alb, art) : 0.0;
                right_n[c] = nr;
            }
            any = false;
            int nl = 0;
            for (int c = 1; c < bins; c++) {
                if (s_bcnt[k][c - 1]) {
                    for (int q = 0; q < 3; q++) {
                        const float l = unord(s_bbox[k][c - 1][q]), r = unord(s_bbox[k][c - 1][3 + q]);
                        alb[q] = any ? (alb[q] < l ? alb[q] : l) : l;
                        art[q] = any ? (art[q] > r ? art[q] : r) : r;
                    }
                    any = true;
                }
                nl += s_bcnt[k][c - 1];
                if (nl == 0 || right_n[c] == 0) continue;
                const double cost = sa_of(alb, art) * nl + right_sa[c] * right_n[c];
                if (cost < best) { best = cost; best_axis = k; best_bin = c; best_nl = nl; }
            }
        }
        s_split[0] = best_axis;
        s_split[1] = best_bin;
        s_split[2] = best_axis < 0 ? cnt / 2 : best_nl;
        if (best_axis >= 0 && (order == 1 || order == 3)) {  // the children's boxes: unions of their bins
            for (int side = 0; side < 2; side++) {
                bool any = false;
                const int c0 = side == 0 ? 0 : best_bin, c1 = side == 0 ? best_bin : bins;
                for (int c = c0; c < c1; c++) {
                    if (!s_bcnt[best_axis][c]) continue;
                    for (int q = 0; q < 3; q++) {
                        const float l = unord(s_bbox[best_axis][c][q]), r = unord(s_bbox[best_axis][c][3 + q]);
                        s_child[side][q] = any ? fminf(s_child[side][q], l) : l;
                        s_child[side][3 + q] = any ? fmaxf(s_child[side][3 + q], r) : r;
                    }
                    any = true;
                }
            }
        }
    }
    __syncthreads();
    const int axis = s_split[0], split_bin = s_split[1], nl = s_split[2];
    const int mid = b + nl;

    // 4. stable partition of idx[b, e) by bin < split_bin (into tmp, then back)
    if (axis >= 0) {
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        int done_l = 0, done_r = 0;
        for (int base = b; base < e; base += kSahBlock) {
            const int i = base + threadIdx.x;
            const bool in = i < e;
            const int j = in ? idx[i] : 0;
            const bool go_left = in && min(bins - 1, (int)((cen[(size_t)j * 3 + axis] - clo[axis]) * scale[axis])) < split_bin;
            const unsigned long long bl = __ballot(go_left), bi = __ballot(in);
            const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
            if (lane == 0) s_wave[wave] = __popcll(bl);
            __syncthreads();
            int before = 0, chunk_l = 0;
            for (int w = 0; w < kSahBlock / 64; w++) {
                if (w < wave) before += s_wave[w];
                chunk_l += s_wave[w];
            }
            const int rank_l = before + __popcll(bl & below);
            const int pos_in_chunk = threadIdx.x;  // elements before this one in the chunk
            const int rank_r = pos_in_chunk - rank_l;
            if (in) {
                if (go_left) tmp[b + done_l + rank_l] = j;
                else tmp[mid + done_r + rank_r] = j;
            }
            const int chunk_n = min(kSahBlock, e - base);
            (void)bi;
            done_l += chunk_l;
            done_r += chunk_n - chunk_l;
            __syncthreads();
        }
        __syncthreads();
        for (int i = b + threadIdx.x; i < e; i += kSahBlock) idx[i] = tmp[i];
    }

    // the children, in the host's preorder child order
    if (threadIdx.x == 0) {
        const int l = atomicAdd(&tree.count[0], 2), r = l + 1;
        bool swap = false;
        if (order == 1 || order == 3) {
            double sl, sr;
            if (axis >= 0) {
                sl = sa_of(&s_child[0][0], &s_child[0][3]);
                sr = sa_of(&s_child[1][0], &s_child[1][3]);
            } else {  // the median split: every centroid equal; boxes by a sequential fold (small and rare)
                float bl_[6], br_[6];
                for (int side = 0; side < 2; side++) {
                    float* o = side == 0 ? bl_ : br_;
                    const int s0 = side == 0 ? b : mid, s1 = side == 0 ? mid : e;
                    for (int q = 0; q < 3; q++) { o[q] = tbox[(size_t)idx[s0] * 6 + q]; o[3 + q] = tbox[(size_t)idx[s0] * 6 + 3 + q]; }
                    for (int i = s0 + 1; i < s1; i++)
                        for (int q = 0; q < 3; q++) {
                            o[q] = fminf(o[q], tbox[(size_t)idx[i] * 6 + q]);
                            o[3 + q] = fmaxf(o[3 + q], tbox[(size_t)idx[i] * 6 + 3 + q]);
                        }
                }
                sl = sa_of(bl_, bl_ + 3);
                sr = sa_of(br_, br_ + 3);
            }
            swap = order == 1 ? sr > sl : sr < sl;
        } else if (order == 2 || order == 4) {
            swap = order == 2 ? (e - mid) > (mid - b) : (e - mid) < (mid - b);
        } else if (order == 5) {
            swap = true;
        }
        tree.left[task.node] = swap ? r : l;
        tree.right[task.node] = swap ? l : r;
        const int t = atomicAdd(&tree.count[1], 2);
        next[t] = SahTask{l, b, mid};
        next[t + 1] = SahTask{r, mid, e};
    }
}

}  // namespace

// PT_BVH_SAH on the device: the host builder's tree (pt_bvh_build_sah, `bins` bins, PT_SAH_ORDER child order),
// flattened on the host (pt_flatten_tree). Same output contract as pt_bvh_build.
extern "C" int pt_bvh_build_sah_device(const pt_triangle* tris, int n, int start_index, int leaf_size, int bins,
                                       pt_bvh_node_device** nodes_out, int* node_num_out, int** leaf_out,
                                       int* leaf_num_out) {
    if (!tris || n <= 0 || leaf_size <= 0 || bins < 2 || bins > kMaxBins || !nodes_out || !node_num_out || !leaf_out ||
        !leaf_num_out)
        return -1;
    const int order_cfg = pt_sah_order();
    const int order = order_cfg == 6 ? 0 : order_cfg;  // 6: reordered on the host (pt_sah_order_by_steps)
    const size_t cap = 2 * (size_t)n;  // nodes of a tree with at least one triangle per leaf
    hipStream_t stream = nullptr;
    void* mem = nullptr;
    std::vector<float> h_box;
    std::vector<int> h_left, h_right, h_begin, h_end, h_idx;
    int nodes = 0;
    auto run = [&]() -> hipError_t {
        SAH_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        size_t off = 0;
        auto take = [&](size_t bytes) { const size_t o = off; off = (off + bytes + 255) & ~(size_t)255; return o; };
        const size_t o_tris = take(sizeof(pt_triangle) * n), o_tbox = take((size_t)n * 24), o_cen = take((size_t)n * 12),
                     o_idx = take((size_t)n * 4), o_tmp = take((size_t)n * 4), o_ta = take(sizeof(SahTask) * cap),
                     o_tb = take(sizeof(SahTask) * cap), o_box = take(cap * 24), o_left = take(cap * 4),
                     o_right = take(cap * 4), o_begin = take(cap * 4), o_end = take(cap * 4), o_count = take(8);
        SAH_HIP(hipMalloc(&mem, off));
        uint8_t* base = static_cast<uint8_t*>(mem);
        pt_triangle* d_tris = reinterpret_cast<pt_triangle*>(base + o_tris);
        float* tbox = reinterpret_cast<float*>(base + o_tbox);
        float* cen = reinterpret_cast<float*>(base + o_cen);
        int* idx = reinterpret_cast<int*>(base + o_idx);
        int* tmp = reinterpret_cast<int*>(base + o_tmp);
        SahTask* ta = reinterpret_cast<SahTask*>(base + o_ta);
        SahTask* tb = reinterpret_cast<SahTask*>(base + o_tb);
        SahTree tree{reinterpret_cast<float*>(base + o_box), reinterpret_cast<int*>(base + o_left),
                     reinterpret_cast<int*>(base + o_right), reinterpret_cast<int*>(base + o_begin),
                     reinterpret_cast<int*>(base + o_end), reinterpret_cast<int*>(base + o_count)};
        SAH_HIP(hipMemcpyAsync(d_tris, tris, sizeof(pt_triangle) * n, hipMemcpyHostToDevice, stream));
        hipLaunchKernelGGL(sah_prepare_kernel, dim3((n + kSahBlock - 1) / kSahBlock), dim3(kSahBlock), 0, stream, d_tris, n,
                           tbox, cen, idx);
        SAH_HIP(hipGetLastError());
        const SahTask root{0, 0, n};
        const int counts[2] = {1, 0};
        SAH_HIP(hipMemcpyAsync(ta, &root, sizeof(root), hipMemcpyHostToDevice, stream));
        SAH_HIP(hipMemcpyAsync(tree.count, counts, sizeof(counts), hipMemcpyHostToDevice, stream));
        int m = 1;
        while (m > 0) {
            SAH_HIP(hipMemsetAsync(tree.count + 1, 0, sizeof(int), stream));
            hipLaunchKernelGGL(sah_level_kernel, dim3(m), dim3(kSahBlock), 0, stream, tbox, cen, idx, tmp, ta, tb, tree,
                               leaf_size, bins, order);
            SAH_HIP(hipGetLastError());
            int got[2] = {0, 0};
            SAH_HIP(hipMemcpyAsync(got, tree.count, sizeof(got), hipMemcpyDeviceToHost, stream));
            SAH_HIP(hipStreamSynchronize(stream));
            if (got[0] > (int)cap) return hipErrorInvalidValue;
            nodes = got[0];
            m = got[1];
            std::swap(ta, tb);
        }
        h_box.resize((size_t)nodes * 6);
        h_left.resize(nodes); h_right.resize(nodes); h_begin.resize(nodes); h_end.resize(nodes); h_idx.resize(n);
        SAH_HIP(hipMemcpyAsync(h_box.data(), tree.box, (size_t)nodes * 24, hipMemcpyDeviceToHost, stream));
        SAH_HIP(hipMemcpyAsync(h_left.data(), tree.left, (size_t)nodes * 4, hipMemcpyDeviceToHost, stream));
        SAH_HIP(hipMemcpyAsync(h_right.data(), tree.right, (size_t)nodes * 4, hipMemcpyDeviceToHost, stream));
        SAH_HIP(hipMemcpyAsync(h_begin.data(), tree.begin, (size_t)nodes * 4, hipMemcpyDeviceToHost, stream));
        SAH_HIP(hipMemcpyAsync(h_end.data(), tree.end, (size_t)nodes * 4, hipMemcpyDeviceToHost, stream));
        SAH_HIP(hipMemcpyAsync(h_idx.data(), idx, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
        SAH_HIP(hipStreamSynchronize(stream));
        return hipSuccess;
    };
    const hipError_t e = run();
    if (mem) (void)hipFree(mem);
    if (stream) (void)hipStreamDestroy(stream);
    if (e != hipSuccess) return -3;
    std::vector<PtTreeNode> tree((size_t)nodes);
    for (int i = 0; i < nodes; i++) {
        PtTreeNode& g = tree[(size_t)i];
        for (int k = 0; k < 3; k++) { g.box.lb[k] = h_box[(size_t)i * 6 + k]; g.box.rt[k] = h_box[(size_t)i * 6 + 3 + k]; }
        g.left = h_left[(size_t)i];
        g.right = h_right[(size_t)i];
        g.leaf = g.left < 0;
        if (g.leaf) {
            g.tris.assign((size_t)leaf_size, -1);
            for (int j = h_begin[(size_t)i]; j < h_end[(size_t)i]; j++) g.tris[(size_t)(j - h_begin[(size_t)i])] = h_idx[(size_t)j] + start_index;
        } else {
            tree[(size_t)g.left].parent = i;
            tree[(size_t)g.right].parent = i;
        }
    }
    if (order_cfg == 6) pt_sah_order_by_steps(tree);
    return pt_flatten_tree(tree, leaf_size, nodes_out, node_num_out, leaf_out, leaf_num_out);
}
