// pt_work.h — work distribution for the persistent kernels.
//
// The reference hands one pixel to one thread and compacts the live list between depths
// (thrust::remove_if + host read-back, Kernel/path_tracer_kernel.cu:767). Here a launch's items
// (pixels for the single-kernel pass, queue slots for the wavefront kernels) live in PT_SHARDS
// regions, region r = slots [r * stride, r * stride + n_r). Each region has one head word that
// waves advance by a chunk with ONE returning atomicAdd: a single head word saturates at ~88
// dequeues per us on MI355X (MI355X_MICROARCH.md "dequeue"), so the heads are sharded per XCD and a
// chunk serves many lanes. A wave starts on the region of its XCD (blockIdx.x % 8 under round-robin
// workgroup placement), so neighbouring pixels — coherent BVH walks — share one L2, and moves on
// to the other regions once its own is drained (work stealing), which balances sky against glass.
#pragma once

#include <hip/hip_runtime.h>

#include "pt_scene.h"

namespace pt {

#define PT_HEAD_STRIDE 32                    // uints between head words: one 128-B line each
#define PT_HEAD_SET (PT_SHARDS * PT_HEAD_STRIDE)  // uints per launch's head set

__device__ __forceinline__ unsigned long long lanes_below(int lane) {
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}
// popcount(m & lanes_below(lane)) of the calling lane: two v_mbcnt, no 64-bit mask held in registers
__device__ __forceinline__ int count_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned int)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned int)m, 0u));
}

// Unit u of this launch's share of the frame -> pixel index (DevTiling: bands of band_rows rows
// dealt round-robin over band_count owners).
__device__ __forceinline__ int unit_to_pixel(const DevTiling& til, unsigned int u) {
    if (til.band_order) {  // bands handed out by cost (pt_set_band_order); its load is waited for in here
        const int row_local = (int)u / til.width;
        const int x = (int)u - row_local * til.width;
        const int band_local = row_local / til.band_rows;
        const int row_in_band = row_local - band_local * til.band_rows;
        const int b = __builtin_nontemporal_load(til.band_order + band_local);
        const int owner = til.band_count > 1 ? til.band_index : 0;  // one owner: band_index is not used (local_bands)
        return ((b * til.band_count + owner) * til.band_rows + row_in_band) * til.width + x;
    }
    if (til.band_count == 1) return (int)u;
    int row_local = (int)u / til.width;
    int x = (int)u - row_local * til.width;
    int band_local = row_local / til.band_rows;
    int row_in_band = row_local - band_local * til.band_rows;
    int y = (band_local * til.band_count + til.band_index) * til.band_rows + row_in_band;
    return y * til.width + x;
}

// Local band of a pixel this launch owns (the inverse of unit_to_pixel's band arithmetic).
__device__ __forceinline__ int pixel_band(const DevTiling& til, int pixel) {
    return pixel / til.width / til.band_rows / til.band_count;
}

struct WorkCursor {
    unsigned int cur, end;  // chunk being handed out (wave-uniform)
    int region;             // region fetched from next
    int left;               // regions not yet found drained
};

__device__ __forceinline__ WorkCursor work_begin() {
    WorkCursor c;
    c.cur = 0;
    c.end = 0;
    c.region = (int)(blockIdx.x % PT_SHARDS);
    c.left = PT_SHARDS;
    return c;
}

// Region sizes of an even split of `units` items (depth 0 / the single-kernel pass).
struct EvenRegions {
    unsigned int units, stride;
    __device__ __forceinline__ unsigned int operator()(int r) const {
        const unsigned int lo = (unsigned int)r * stride;
        return units > lo ? (units - lo < stride ? units - lo : stride) : 0u;
    }
};

// Region sizes of a depth >= 1 queue: the append counters of its shards.
struct QueueRegions {
    const unsigned int* counts;
    __device__ __forceinline__ unsigned int operator()(int r) const { return counts[r]; }
};

// Next non-empty chunk of at most `chunk` items into `c`; false once every region is drained.
// Called by the whole wave with uniform arguments.
template <class Sizes>
__device__ __forceinline__ bool work_fetch(unsigned int* heads, unsigned int stride, const Sizes& size_of,
                                           unsigned int chunk, WorkCursor& c) {
    while (c.left > 0) {
        unsigned int off = 0;
        if ((threadIdx.x & 63) == 0) off = atomicAdd(heads + c.region * PT_HEAD_STRIDE, chunk);
        off = (unsigned int)__builtin_amdgcn_readfirstlane((int)off);
        const unsigned int n = size_of(c.region);
        if (off < n) {
            c.cur = (unsigned int)c.region * stride + off;
            c.end = c.cur + (n - off < chunk ? n - off : chunk);
            return true;
        }
        c.region = (c.region + 1) & (PT_SHARDS - 1);
        c.left--;
    }
    return false;
}

// Hands one item to every lane in `want_mask`, in lane order, spilling into a freshly fetched
// chunk when the current one runs out. chunk == 0 fetches exactly the shortfall (no reserve held
// by the wave: the end-of-launch tail is then one path, not one chunk, per lane). Returns this lane's item or ~0u (none yet, or none left:
// `drained` is set once every region is empty). Called by the whole wave.
template <class Sizes>
__device__ __forceinline__ unsigned int work_take(unsigned int* heads, unsigned int stride, const Sizes& size_of,
                                                  unsigned int chunk, unsigned long long want_mask, bool want,
                                                  unsigned long long lanes_lt, WorkCursor& c, bool& drained) {
    const unsigned int taken = (unsigned int)__popcll(want_mask);
    const unsigned int rank = (unsigned int)__popcll(want_mask & lanes_lt);
    const unsigned int avail = c.end - c.cur;
    unsigned int u = ~0u;
    if (want && rank < avail) u = c.cur + rank;
    if (taken <= avail) {
        c.cur += taken;
        return u;
    }
    const unsigned int rest = taken - avail;
    if (!work_fetch(heads, stride, size_of, chunk ? chunk : rest, c)) {
        c.cur = c.end;
        drained = true;
        return u;
    }
    const unsigned int got = c.end - c.cur;
    if (want && rank >= avail && rank - avail < got) u = c.cur + (rank - avail);
    c.cur += rest < got ? rest : got;
    return u;
}

}  // namespace pt
