// pt_wavefront.hip — the wavefront schedule of one pass (default path).
//
// The reference runs, per depth, one thread per live pixel through BOTH the BVH walk and the
// shading (trace_ray_kernel, Kernel/path_tracer_kernel.cu:381-625), then compacts the live list
// with thrust::remove_if and a host read-back (:767). Measured on MI355X, that shape in one kernel
// keeps only ~6 of 64 lanes busy per VALU instruction: walk lengths differ per ray and the shading
// branches diverge. Here each depth is two kernels over a dense ray queue:
//
//   extend_kernel  persistent BVH walk. A lane owns one ray at a time and advances it by one node
//                  per loop iteration; when its ray finishes, the wave ballots the idle lanes and
//                  refills them from the wave's own contiguous range of the queue (per-lane ray
//                  replacement, no atomics), so lanes stay busy until the range drains. Writes a
//                  16-B hit record per ray.
//   shade_kernel   medium / material / Fresnel / bounce for every queued ray, radiance into the
//                  pixel's state, and the live rays appended to the next depth's queue by a wave
//                  ballot + one atomicAdd on one of 8 shard counters (the reference's
//                  thread_shrink, without the host).
//   finalize_kernel  the per-pass clamp + running sum + gamma/8-bit (pixel_256_transform_..., :627-682).
//
// Depth 0 generates camera rays inside extend_kernel (generate_ray_kernel, :299-379). Per-ray
// arithmetic is the same code as the single-kernel path (pt_path.h), so results are bit-identical.
#include <cstdlib>

#include "pt_kernels.h"

namespace pt {

__device__ __forceinline__ void wave_reduce_add(unsigned long long* dst, unsigned long long v, int lane) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0 && v) atomicAdd(dst, v);
}

// Walk state of the ray a lane owns (path_tracer_kernel.cu:418-454 unrolled into single steps).
struct Walk {
    v3 o, d, inv;
    int pos, end, mesh;
    float mt, mt1, mt2;  // closest hit in the current mesh (intersect_triangle_mesh_bvh's min_*)
    int mtri;
    Hit best;            // closest hit over spheres and finished meshes
};

// Finish meshes whose walk is complete; false once every mesh is done.
__device__ __forceinline__ bool walk_advance(const DevScene& sc, Walk& w) {
    while (w.pos == w.end) {
        if (w.mtri >= 0 && w.mt < w.best.t && w.mt > 0.0f) {  // :445
            w.best.t = w.mt; w.best.t1 = w.mt1; w.best.t2 = w.mt2; w.best.prim = w.mtri; w.best.type = 2;
        }
        w.mesh++;
        if (w.mesh >= sc.mesh_num) return false;
        int2 r = sc.mesh_range[w.mesh];
        w.pos = r.x; w.end = r.y;
        w.mt = __builtin_inff(); w.mtri = -1;
    }
    return true;
}

template <bool GEN, bool LEAF1, bool STATS>
__global__ __launch_bounds__(PT_BLOCK) void extend_kernel(const LaunchParams* __restrict__ P, int depth, int pass,
                                                          int refill, int chunk) {
    const DevScene& sc = P->sc;
    const DevWave& W = P->wave;
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = lanes_below(lane);
    const unsigned int S = (unsigned int)W.seg_cap;
    const EvenRegions even{(unsigned int)P->til.unit_count, S};
    const QueueRegions queued{W.counters + depth * PT_SHARDS};
    unsigned int* heads = W.heads + (size_t)(2 * depth) * PT_HEAD_SET;
    WorkCursor cursor = work_begin();
    bool drained = false;
    float4* q_o = W.q_o[depth & 1];
    float4* q_d = W.q_d[depth & 1];
    const __amdgpu_buffer_rsrc_t rn = make_rsrc(sc.nodes, sc.node_count * 32);
    const __amdgpu_buffer_rsrc_t rt = make_rsrc(sc.tri_geom, sc.tri_count * 48);
    const int32_t hseed = hash_pt(pass);

    Walk w;
    unsigned int ray = 0;  // queue slot of the ray this lane walks
    bool active = false, exhausted = false;
    unsigned long long c_nodes = 0, c_tris = 0;

    while (true) {
        const bool want = !active && !exhausted;
        const unsigned long long idle = __ballot(want);
        if (idle && (__popcll(idle) >= refill || __ballot(active) == 0)) {
            unsigned int u;
            if (GEN) u = work_take(heads, S, even, (unsigned int)chunk, idle, want, lt, cursor, drained);
            else u = work_take(heads, S, queued, (unsigned int)chunk, idle, want, lt, cursor, drained);
            if (want) {
                if (u != ~0u) {
                    ray = u;
                    if (GEN) {
                        // depth 0: slot == unit (EvenRegions cut the units into the same regions)
                        const int pixel = unit_to_pixel(P->til, ray);
                        PathState ps;
                        generate_path(P->cam, P->cfg, pixel, hseed, &ps);
                        w.o = ps.o; w.d = ps.d;
                        q_o[ray] = make_float4(w.o.x, w.o.y, w.o.z, __int_as_float(pixel));
                        q_d[ray] = make_float4(w.d.x, w.d.y, w.d.z, 0.0f);
                    } else {
                        float4 a = q_o[ray], b = q_d[ray];
                        w.o = mk3(a.x, a.y, a.z); w.d = mk3(b.x, b.y, b.z);
                    }
                    // spheres by brute force (:431-441)
                    w.best.t = __builtin_inff(); w.best.t1 = __builtin_inff(); w.best.t2 = __builtin_inff();
                    w.best.type = 0; w.best.prim = -1;
                    for (int i = 0; i < sc.sphere_num; i++) {
                        float t;
                        if (sphere_t(sc.spheres[2 * i], w.o, w.d, &t) && t < w.best.t && t > 0.0f) {
                            w.best.t = t; w.best.prim = i; w.best.type = 1;
                        }
                    }
                    w.inv = 1.0f / w.d;
                    w.mesh = -1; w.pos = 0; w.end = 0; w.mtri = -1;
                    active = walk_advance(sc, w);
                    if (!active) W.hit[ray] = make_float4(w.best.t, w.best.t1, w.best.t2,
                                                          __int_as_float((w.best.prim << 2) | w.best.type));
                } else if (drained) {
                    exhausted = true;
                }
            }
        }
        if (__ballot(!exhausted) == 0) break;
        if (!active) continue;

        // one node of the stackless preorder walk (:113-150)
        const float4 lo = bload(rn, w.pos * 32), hi4 = bload(rn, w.pos * 32 + 16);
        if (STATS) c_nodes++;
        float entry;
        if (box_hit(lo, hi4, w.o, w.inv, &entry) && entry <= w.mt) {
            const int slot_or_tri = __float_as_int(hi4.w);
            if (slot_or_tri >= 0) {
                if (LEAF1) {
                    float t, t1, t2;
                    if (STATS) c_tris++;
                    const int tri = slot_or_tri;
                    float4 a = bload(rt, tri * 48), b = bload(rt, tri * 48 + 16), c = bload(rt, tri * 48 + 32);
                    if (triangle_test(a, b, c, w.o, w.d, &t, &t1, &t2) && t > 0.0f && t < w.mt) {
                        w.mt = t; w.mt1 = t1; w.mt2 = t2; w.mtri = tri;
                    }
                } else {
                    for (int i = 0; i < sc.leaf_size; i++) {
                        const int tri = sc.leaf_tris[slot_or_tri + i];
                        if (tri == -1) break;
                        float t, t1, t2;
                        if (STATS) c_tris++;
                        float4 a = bload(rt, tri * 48), b = bload(rt, tri * 48 + 16), c = bload(rt, tri * 48 + 32);
                        if (triangle_test(a, b, c, w.o, w.d, &t, &t1, &t2) && t > 0.0f && t < w.mt) {
                            w.mt = t; w.mt1 = t1; w.mt2 = t2; w.mtri = tri;
                        }
                    }
                }
            }
            w.pos++;
        } else {
            w.pos = __float_as_int(lo.w);
        }
        if (w.pos == w.end && !walk_advance(sc, w)) {
            W.hit[ray] = make_float4(w.best.t, w.best.t1, w.best.t2, __int_as_float((w.best.prim << 2) | w.best.type));
            active = false;
        }
    }
    if (STATS) {
        wave_reduce_add(&P->out.stats[1], c_nodes, lane);
        wave_reduce_add(&P->out.stats[2], c_tris, lane);
    }
}

template <bool FIRST, bool LAST, bool STATS>
__global__ __launch_bounds__(PT_BLOCK) void shade_kernel(const LaunchParams* __restrict__ P, int depth, int pass,
                                                         int chunk) {
    const DevScene& sc = P->sc;
    const DevConfig& cfg = P->cfg;
    const DevWave& W = P->wave;
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = lanes_below(lane);
    const unsigned int S = (unsigned int)W.seg_cap;
    const EvenRegions even{(unsigned int)P->til.unit_count, S};
    const QueueRegions queued{W.counters + depth * PT_SHARDS};
    unsigned int* heads = W.heads + (size_t)(2 * depth + 1) * PT_HEAD_SET;
    WorkCursor cursor = work_begin();
    const float4* q_o = W.q_o[depth & 1];
    const float4* q_d = W.q_d[depth & 1];
    const int32_t hseed = hash_pt(pass);
    unsigned long long segs = 0;
    Counters ctr = {0u, 0u, 0u, 0u, 0u, 0u};

    // Survivors of region k go to shard k of the next queue, so a shard never holds more rays than
    // its depth-0 region (<= S = seg_cap) whichever waves shade them.
    while (FIRST ? work_fetch(heads, S, even, (unsigned int)chunk, cursor)
                 : work_fetch(heads, S, queued, (unsigned int)chunk, cursor)) {
        const int shard = cursor.region;
        unsigned int* out_count = W.counters + (depth + 1) * PT_SHARDS + shard;
        float4* out_o = W.q_o[(depth + 1) & 1] + (size_t)shard * S;
        float4* out_d = W.q_d[(depth + 1) & 1] + (size_t)shard * S;
        for (unsigned int base = cursor.cur; base < cursor.end; base += 64) {
            const unsigned int slot = base + (unsigned int)lane;
            const bool valid = slot < cursor.end;
            bool alive = false;
            PathState ps;
            int pixel = 0;
            if (valid) {
                const float4 a = q_o[slot], b = q_d[slot], hh = W.hit[slot];
                pixel = __float_as_int(a.w);
                ps.o = mk3(a.x, a.y, a.z);
                ps.d = mk3(b.x, b.y, b.z);
                if (FIRST) {
                    ps.thr = mk3(1.0f, 1.0f, 1.0f);
                    ps.rad = mk3(0.0f, 0.0f, 0.0f);
                    ps.medium = -1;
                } else {
                    const float4 t = W.st_thr[pixel], r = W.st_rad[pixel];
                    ps.thr = mk3(t.x, t.y, t.z);
                    ps.medium = __float_as_int(t.w);
                    ps.rad = mk3(r.x, r.y, r.z);
                }
                Hit h;
                h.t = hh.x; h.t1 = hh.y; h.t2 = hh.z;
                const int code = __float_as_int(hh.w);
                h.type = code & 3;
                h.prim = code >> 2;
                alive = shade_hit<STATS>(sc, cfg, depth, path_seed(hseed, pixel), &ps, h, &ctr);
                W.st_rad[pixel] = make_float4(ps.rad.x, ps.rad.y, ps.rad.z, 0.0f);
                if (!LAST && alive)
                    W.st_thr[pixel] = make_float4(ps.thr.x, ps.thr.y, ps.thr.z, __int_as_float(ps.medium));
                segs++;
            }
            if (!LAST) {
                const unsigned long long m = __ballot(valid && alive);
                if (m) {
                    const int leader = __ffsll((long long)m) - 1;
                    unsigned int qb = 0;
                    if (lane == leader) qb = atomicAdd(out_count, (unsigned int)__popcll(m));
                    qb = __shfl(qb, leader);
                    if (valid && alive) {
                        const unsigned int q = qb + (unsigned int)__popcll(m & lt);
                        out_o[q] = make_float4(ps.o.x, ps.o.y, ps.o.z, __int_as_float(pixel));
                        out_d[q] = make_float4(ps.d.x, ps.d.y, ps.d.z, 0.0f);
                    }
                }
            }
        }
    }
    wave_reduce_add(&P->out.stats[0], segs, lane);
    if (STATS) {
        wave_reduce_add(&P->out.stats[3], ctr.hit_mesh, lane);
        wave_reduce_add(&P->out.stats[4], ctr.hit_sphere, lane);
        wave_reduce_add(&P->out.stats[5], ctr.miss, lane);
        wave_reduce_add(&P->out.stats[6], ctr.scatter, lane);
    }
}

// pixel_256_transform_gamma_corrected_kernel (:627-682) over the pixels this launch owns.
__global__ __launch_bounds__(PT_BLOCK) void finalize_kernel(const LaunchParams* __restrict__ P, int pass, int write_u8,
                                                            int traced) {
    const unsigned int u = blockIdx.x * PT_BLOCK + threadIdx.x;
    if (u >= (unsigned int)P->til.unit_count) return;
    const DevConfig& cfg = P->cfg;
    const int pixel = unit_to_pixel(P->til, u);
    v3 rad = mk3(0.0f, 0.0f, 0.0f);
    if (traced) {
        const float4 r = P->wave.st_rad[pixel];
        rad = mk3(r.x, r.y, r.z);
    }
    float* img = P->out.image + (size_t)pixel * 3;
    const v3 c = clamp3(rad, 0.0f, (float)cfg.max_depth * 2.0f);
    v3 sum;
    if (pass != 1) sum = mk3(img[0], img[1], img[2]) + c;
    else sum = c;
    img[0] = sum.x; img[1] = sum.y; img[2] = sum.z;
    if (write_u8 && P->out.image256) store_u8(cfg, sum, pass, P->out.image256 + (size_t)pixel * 3);
}

// ---- launchers ------------------------------------------------------------------------------
using ExtendFn = void (*)(const LaunchParams*, int, int, int, int);
using ShadeFn = void (*)(const LaunchParams*, int, int, int);

static ExtendFn extend_fn(bool gen, bool leaf1, bool stats) {
    if (gen) {
        if (leaf1) return stats ? extend_kernel<true, true, true> : extend_kernel<true, true, false>;
        return stats ? extend_kernel<true, false, true> : extend_kernel<true, false, false>;
    }
    if (leaf1) return stats ? extend_kernel<false, true, true> : extend_kernel<false, true, false>;
    return stats ? extend_kernel<false, false, true> : extend_kernel<false, false, false>;
}

static ShadeFn shade_fn(bool first, bool last, bool stats) {
    if (stats) {
        if (first) return last ? shade_kernel<true, true, true> : shade_kernel<true, false, true>;
        return last ? shade_kernel<false, true, true> : shade_kernel<false, false, true>;
    }
    if (first) return last ? shade_kernel<true, true, false> : shade_kernel<true, false, false>;
    return last ? shade_kernel<false, true, false> : shade_kernel<false, false, false>;
}

static int occupancy_grid(const void* fn) {
    int dev = 0, cus = 0, blocks = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, PT_BLOCK, 0) != hipSuccess || blocks <= 0) blocks = 4;
    if (cus <= 0) cus = 256;
    return cus * blocks;
}

int wave_refill_threshold() {
    static int r = [] {
        const char* e = getenv("PT_REFILL");
        int v = e ? atoi(e) : 16;
        return v < 1 ? 1 : (v > 64 ? 64 : v);
    }();
    return r;
}

hipError_t launch_extend(const LaunchParams* P, bool gen, bool leaf1, bool stats, int depth, int pass, hipStream_t s) {
    ExtendFn fn = extend_fn(gen, leaf1, stats);
    static int grid[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int& g = grid[(gen ? 4 : 0) + (leaf1 ? 2 : 0) + (stats ? 1 : 0)];
    if (g == 0) g = occupancy_grid((const void*)fn);
    int refill = wave_refill_threshold();
    static const int chunk = env_int("PT_CHUNK_EXTEND", 0, 0, 4096);
    int ck = chunk;
    void* args[] = {(void*)&P, &depth, &pass, &refill, &ck};
    hipError_t e = hipLaunchKernel((const void*)fn, dim3(g), dim3(PT_BLOCK), args, 0, s);
    return e != hipSuccess ? e : hipGetLastError();
}

// One grid for every shade variant: the shard capacity (pt_runtime.cpp) is sized from it.
int shade_grid_waves() {
    static int waves = [] {
        int g = 0;
        for (int v = 0; v < 8; v++) {
            int x = occupancy_grid((const void*)shade_fn(v & 4, v & 2, v & 1));
            g = x > g ? x : g;
        }
        return g * (PT_BLOCK / 64);
    }();
    return waves;
}

hipError_t launch_shade(const LaunchParams* P, bool first, bool last, bool stats, int depth, int pass, hipStream_t s) {
    ShadeFn fn = shade_fn(first, last, stats);
    const int g = shade_grid_waves() / (PT_BLOCK / 64);
    static const int chunk = env_int("PT_CHUNK_SHADE", 256, 64, 4096);
    int ck = chunk;
    void* args[] = {(void*)&P, &depth, &pass, &ck};
    hipError_t e = hipLaunchKernel((const void*)fn, dim3(g), dim3(PT_BLOCK), args, 0, s);
    return e != hipSuccess ? e : hipGetLastError();
}

hipError_t launch_finalize(const LaunchParams* P, int units, int pass, int write_u8, int traced, hipStream_t s) {
    if (units <= 0) return hipSuccess;
    int grid = (units + PT_BLOCK - 1) / PT_BLOCK;
    hipLaunchKernelGGL(finalize_kernel, dim3(grid), dim3(PT_BLOCK), 0, s, P, pass, write_u8, traced);
    return hipGetLastError();
}

}  // namespace pt
