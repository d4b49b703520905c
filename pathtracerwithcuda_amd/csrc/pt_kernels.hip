// pt_kernels.hip — HIP kernels of the radiance loop for gfx950.
//
// Reference structure (Kernel/path_tracer_kernel.cu:685-780): per pass, init_data_kernel ->
// generate_ray_kernel -> max_depth x (trace_ray_kernel + thrust::remove_if compaction with a
// host read-back of the live count) -> pixel_256_transform_gamma_corrected_kernel.
//
// Here one pass is ONE persistent launch. Each 64-lane wave owns up to 64 paths held entirely
// in registers (the reference round-trips 76 B/pixel of path state through memory every depth).
// A lane whose path terminates (killed, escaped, or max depth reached) writes its pixel's
// running sum and 8-bit value and is refilled from a global pixel counter: the wave ballots the
// lanes that need work, the first such lane takes popc(ballot) pixels with ONE atomicAdd, and
// each lane takes its rank among them (mbcnt). That is the reference's thread_shrink compaction
// (stable remove_if of dead pixels) done in-register, per wave, with no host synchronisation.
// Results do not depend on the schedule: every random draw is seeded by (pass, pixel, depth)
// (path_tracer_kernel.cu:324,415) and a pixel's passes are ordered by the launch sequence.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "pt_kernels.h"

namespace pt {

// PT_DUP (diagnostic builds only, -DPT_DUP=n via PT_EXTRA_FLAGS into a separate PT_LIBDIR): run one
// phase twice on opaque copies of its inputs and discard the copy's result, so that the PMC
// difference SQ_INSTS_VALU(dup) - SQ_INSTS_VALU(normal) is the VALU count of that phase over the
// same dynamic paths (1 shading, 2 box stage, 3 triangle stage, 4 path generation). The product
// build has PT_DUP 0 and none of this code.
#ifndef PT_DUP
#define PT_DUP 0
#endif
#ifndef PT_MESH_SITE
#define PT_MESH_SITE 1
#endif
// PT_NEXT_MESH: mesh changes read the LDS next-mesh table (start_mesh_next); 0: the mesh loop
#ifndef PT_NEXT_MESH
#define PT_NEXT_MESH 1
#endif
// PT_ROOT_SKIP: segments test every mesh's root box at their start and skip the meshes they miss
#ifndef PT_PROF_MESH
#define PT_PROF_MESH 0
#endif
#ifndef PT_ROOT_SKIP
#define PT_ROOT_SKIP 1
#endif
// PT_KEEP_PARKED: lanes parked on a leaf stay parked across a round's end (and a shading batch) instead of
// the round's last walk step testing their triangles in a forced batch; the next round re-issues their
// triangle loads (experiment: fewer, fuller triangle batches)
#ifndef PT_KEEP_PARKED
#define PT_KEEP_PARKED 0
#endif
// PT_DEFER: pass_kernel_u lanes walk on past a passing leaf and test its triangle later (pt_path.h,
// "deferred leaves"), so triangle batches wait for more lanes without parking them
#ifndef PT_DEFER
#define PT_DEFER 0
#endif
template <class T>
__device__ __forceinline__ void opaque(T& x) {
    int* p = reinterpret_cast<int*>(&x);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); i++) asm volatile("" : "+v"(p[i]));
}


// A copy of *p read through the constant address space: the loads are known not to alias the
// kernel's stores, so a wave-uniform p becomes scalar loads into SGPRs (s_load_dwordx*), not
// vector loads that cost VGPRs and vector-memory issue slots.
template <class T>
__device__ __forceinline__ T load_const(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(4))) const T ConstT;
    const ConstT* c = (const ConstT*)(unsigned long long)p;
    return *c;
#else
    return *p;
#endif
}

// MINW = minimum waves per SIMD requested from the register allocator; the persistent loop is
// latency-bound, so occupancy is the first-order knob.
//
// One launch renders 2^batch_log2 consecutive passes (first_pass ...). Work unit u is pass
// first_pass + (u & (B-1)) of local pixel u >> batch_log2: the passes of one pixel sit in adjacent
// lanes, so their primary rays (same pixel, different jitter) walk the same BVH nodes together.
// With B == 1 a finished path accumulates into the image directly; with B > 1 it stores its clamped
// radiance in pass_rad[u] and accumulate_kernel sums the passes in pass order afterwards, so the
// running sum is bit-identical to one launch per pass.
template <bool LEAF1, bool STATS, int MINW, bool QN>
__global__ __launch_bounds__(PT_BLOCK, MINW) void pass_kernel(const LaunchParams* __restrict__ params, int first_pass,
                                                              int write_u8, int chunk, int batch_log2) {
    const int lane = threadIdx.x & 63;
    const LaunchParams* P0 = params;
    const DevConfig& cfg0 = P0->cfg;
    const DevOutput& out0 = P0->out;
    const float clamp_hi = (float)cfg0.max_depth * 2.0f;
    const unsigned long long lane_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    PathState ps;
    unsigned int unit = 0;
    int32_t pseed = 0;
    int depth = 0;
    bool need = true;   // lane wants a new path
    bool done = false;  // no work left for this lane
    unsigned long long segments = 0;
    Counters ctr = {0u, 0u, 0u, 0u, 0u, 0u};
    unsigned long long csum[6] = {0, 0, 0, 0, 0, 0};
    // (pixel, pass) units in PT_SHARDS regions handed out by per-XCD head words (pt_work.h)
    const unsigned int units = (unsigned int)P0->til.unit_count << batch_log2;
    const EvenRegions regions{units, (units + PT_SHARDS - 1) / PT_SHARDS};
    WorkCursor cursor = work_begin();
    bool drained = false;

    while (true) {
        // The launch parameters are re-read every iteration (scalar loads, K$ hits) rather than held
        // in registers across the whole loop: the empty asm hides the pointer from loop-invariant
        // code motion; readfirstlane restores its uniformity (asm results count as divergent), and
        // the constant-address-space read makes the loads scalar (s_load into SGPRs).
        const LaunchParams* P = params;
        asm volatile("" : "+s"(P));
        P = uniform_ptr(P);
        const DevScene sc = load_const(&P->sc);
        const DevConfig cfg = load_const(&P->cfg);
        const DevTiling til = load_const(&P->til);
        const DevOutput out = load_const(&P->out);
        const bool want = need && !done;
        const unsigned long long need_mask = __ballot(want);
        if (need_mask) {
            const unsigned int u = work_take(out.fetch, regions.stride, regions, (unsigned int)chunk, need_mask, want,
                                             lane_lt, cursor, drained);
            if (want) {
                if (u != ~0u) {
                    need = false;
                    unit = u;
                    const int pixel = unit_to_pixel(til, u >> batch_log2);
                    const int32_t hseed = hash_pt(first_pass + (int)(u & ((1u << batch_log2) - 1u)));
                    const DevCamera cam = load_const(&P->cam);
                    generate_path(cam, cfg, pixel, hseed, &ps);
                    pseed = path_seed(hseed, pixel);
                    depth = 0;
                } else if (drained) {
                    done = true;
                }
            }
        }
        if (!__any(!done)) break;
        if (!done && !need) {  // a lane still waiting for a unit (chunk ran short) has no path yet
            bool alive = false;
            if (depth < cfg.max_depth) {
                alive = trace_step<LEAF1, STATS, QN>(sc, cfg, depth, pseed, &ps, &ctr);
                depth++;
                segments++;
                if (STATS) {
                    csum[0] += ctr.nodes; csum[1] += ctr.tris; csum[2] += ctr.hit_mesh;
                    csum[3] += ctr.hit_sphere; csum[4] += ctr.miss; csum[5] += ctr.scatter;
                    ctr = Counters{0u, 0u, 0u, 0u, 0u, 0u};
                }
            }
            if (!alive || depth >= cfg.max_depth) {
                // pixel_256_transform_gamma_corrected_kernel (:644-680) for this (pixel, pass)
                const v3 c = clamp3(ps.rad, 0.0f, clamp_hi);
                if (batch_log2 == 0) {
                    const int pixel = unit_to_pixel(til, unit);
                    float* img = out.image + (size_t)pixel * 3;
                    v3 sum;
                    if (first_pass != 1) sum = mk3(img[0], img[1], img[2]) + c;
                    else sum = c;
                    img[0] = sum.x; img[1] = sum.y; img[2] = sum.z;
                    if (write_u8 && out.image256) store_u8(cfg, sum, first_pass, out.image256 + (size_t)pixel * 3);
                } else {
                    float* pr = out.pass_rad + (size_t)unit * 3;
                    pr[0] = c.x; pr[1] = c.y; pr[2] = c.z;
                }
                need = true;
            }
        }
    }

    // ray-segment count = sum of the live counts thread_shrink would return (metric numerator)
    unsigned long long s = segments;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (STATS) {
#pragma unroll
        for (int k = 0; k < 6; k++)
            for (int off = 32; off > 0; off >>= 1) csum[k] += __shfl_xor(csum[k], off);
    }
    if (lane == 0) {
        atomicAdd(&out0.stats[0], s);
        if (STATS) {
#pragma unroll
            for (int k = 0; k < 6; k++) atomicAdd(&out0.stats[1 + k], csum[k]);
        }
    }
}

// ---- pass_kernel_u: the same pass with walks and shading interleaved per lane -------------------
// pass_kernel runs one whole trace step (spheres, every mesh walk, shading) per loop iteration for
// all lanes together, so a wave walks as long as its longest walk while finished lanes idle. Here a
// lane is a small state machine: WALK (one BVH node per step of the mesh in flight, then the next
// mesh), READY (closest hit known) and, for the wave, a SHADE step that runs shade_hit for every
// READY lane at once — taken when no lane is walking or at least shade_min lanes are ready — after
// which an ended path takes a new pixel and a surviving one starts its next segment (spheres, mesh 0):
// both in the next round's refill, so one begin_segment serves new and surviving paths together
// (+2.5 % over starting survivors inside the shading batch, profiles/r02/onesite.txt). Every lane still computes exactly the reference sequence for its path (same node order,
// same tests, same draws keyed by (pass, pixel, depth)); only the interleaving between lanes changes.
enum : int { LANE_WANT = 0, LANE_WALK = 1, LANE_READY = 2, LANE_DONE = 3, LANE_TRI = 4, LANE_NEW = 5 };

// Starts the walk of the first mesh at or after `mesh` with a non-empty node range. The ranges of the
// first PT_LDS_MESHES meshes come from the workgroup's LDS copy (lds_mesh, filled at kernel start), the
// rest from global memory. `wide`: the lane walks the wide records (pt_path.h walk_wide): its position is
// the mesh's wide start (lds_wroot / mesh_wide) and `end` is -1, the wide walk's end marker.
#define PT_LDS_MESHES 64
typedef int i32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bool start_mesh(const DevScene& sc, const int2* lds_mesh, const int* lds_wroot, bool wide,
                                           int& mesh, MeshWalk& w) {
    while (mesh < sc.mesh_num) {
        int2 r;
        if (wide) {
            int root;
            if (mesh < PT_LDS_MESHES) {
                root = lds_wroot[mesh];
            } else {
                root = __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(sc.mesh_wide, sc.mesh_num * 4), mesh * 4, 0, 0);
            }
            r.x = root; r.y = root == -1 ? -1 : -2;  // -1: empty mesh
        } else if (mesh < PT_LDS_MESHES) {
            r = lds_mesh[mesh];
        } else {  // a buffer load (not a pointer select that would turn both into flat loads)
            const i32x2 v = __builtin_bit_cast(i32x2, __builtin_amdgcn_raw_buffer_load_b64(
                make_rsrc(sc.mesh_range, sc.mesh_num * 8), mesh * 8, 0, 0));
            r.x = v.x; r.y = v.y;
        }
        if (r.x != r.y) {
            w.pos = r.x; w.end = wide ? -1 : r.y;
            w.t = __builtin_inff(); w.t1 = 0.0f; w.t2 = 0.0f; w.tri = -1;
            return true;
        }
        mesh++;
    }
    return false;
}

// start_mesh for scenes of at most PT_LDS_MESHES meshes walking the binary nodes: lds_next[m] holds the
// range and index of the first non-empty mesh at or after m (index mesh_num and an empty range: none
// left), built at kernel start. One LDS read and no loop: a mesh change in a walk step then waits only
// on LDS, not on the wave's outstanding vector loads (the looping version's mixed LDS / buffer-load
// path made it wait for every one, parked lanes' triangle prefetches included).
__device__ __forceinline__ bool start_mesh_next(const int4* lds_next, int& mesh, MeshWalk& w) {
    const int4 e = lds_next[mesh];
    mesh = e.z;
    if (e.x == e.y) return false;
    w.pos = e.x; w.end = e.y;
    w.t = __builtin_inff(); w.t1 = 0.0f; w.t2 = 0.0f; w.tri = -1;
    return true;
}

// Start of one trace_ray_kernel invocation (path_tracer_kernel.cu:418-454): brute-force spheres into
// the closest hit, then the walk of mesh 0. WIDE scenes: a lane whose 1/d is finite walks the wide
// records, any other the binary nodes (walk_wide's exactness needs a finite 1/d).
template <bool WIDE>
__device__ __forceinline__ int begin_segment(const DevScene& sc, const int2* lds_mesh, const PathState& ps, v3& inv,
                                             Hit& h, MeshWalk& w, int& mesh) {
    h.t = __builtin_inff(); h.t1 = __builtin_inff(); h.t2 = __builtin_inff();
    h.type = 0; h.prim = -1;
    for (int i = 0; i < sc.sphere_num; i++) {
        float t;
        if (sphere_t(sc.spheres[2 * i], ps.o, ps.d, &t) && t < h.t && t > 0.0f) {
            h.t = t; h.prim = i; h.type = 1;
        }
    }
    if (sc.first_mesh >= sc.mesh_num) return LANE_READY;  // (start_mesh from mesh 0, resolved on the host)
    inv = mk3(rcp_exact(ps.d.x), rcp_exact(ps.d.y), rcp_exact(ps.d.z));  // == 1.0f / d
    mesh = sc.first_mesh;
    const bool wide = WIDE && __builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z);
    if (wide) {
        w.pos = sc.first_wide; w.end = -1;
    } else {
        w.pos = sc.first_range.x; w.end = sc.first_range.y;
    }
    w.t = __builtin_inff(); w.t1 = 0.0f; w.t2 = 0.0f; w.tri = -1;
    return LANE_WALK;
}

// ---- root boxes at segment start (pass_kernel_u, binary walk, at most PT_ROOT_MESHES meshes) ----------
// Each mesh's walk starts at its root with a local min_t of infinity (intersect_triangle_mesh_bvh,
// :113-150), so a ray whose slab test fails on a mesh's root box gets nothing from that mesh. The roots of
// the first PT_ROOT_MESHES meshes are kept in LDS; a segment tests them all at its start and walks only the
// meshes whose root passes, starting below a passing internal root (the test there would repeat the same
// test with the same infinite min_t). `mesh` then holds the mesh being walked in bits 0-7 and the meshes
// still to walk as a bit mask from bit 8 on (bit 8 + i: mesh i), so the skip costs no register.
#define PT_ROOT_MESHES 24
__device__ __forceinline__ void root_walk_start(const int2* lds_mesh, const float4* lds_root, int m, MeshWalk& w) {
    const int2 r = lds_mesh[m];
    w.pos = f2i(lds_root[2 * m + 1].w) < 0 ? r.x + 1 : r.x;  // below an internal root, at a leaf root
    w.end = r.y;
    w.t = __builtin_inff(); w.t1 = 0.0f; w.t2 = 0.0f; w.tri = -1;
}
__device__ __forceinline__ int begin_segment_roots(const DevScene& sc, const int2* lds_mesh, const float4* lds_root,
                                                   const PathState& ps, v3& inv, Hit& h, MeshWalk& w, int& mesh) {
    h.t = __builtin_inff(); h.t1 = __builtin_inff(); h.t2 = __builtin_inff();
    h.type = 0; h.prim = -1;
    for (int i = 0; i < sc.sphere_num; i++) {
        float t;
        if (sphere_t(sc.spheres[2 * i], ps.o, ps.d, &t) && t < h.t && t > 0.0f) {
            h.t = t; h.prim = i; h.type = 1;
        }
    }
    if (sc.first_mesh >= sc.mesh_num) return LANE_READY;
    inv = mk3(rcp_exact(ps.d.x), rcp_exact(ps.d.y), rcp_exact(ps.d.z));  // == 1.0f / d
    unsigned int todo = 0;
    for (int i = sc.first_mesh; i < sc.mesh_num; i++) {  // wave-uniform loop, broadcast LDS reads
        const int2 r = lds_mesh[i];
        if (r.x == r.y) continue;
        float entry;
        if (box_hit(lds_root[2 * i], lds_root[2 * i + 1], ps.o, inv, &entry) && entry <= __builtin_inff())
            todo |= 1u << i;
    }
    if (!todo) return LANE_READY;
    const int m = __builtin_ctz(todo);
    mesh = m | (int)((todo & (todo - 1u)) << 8);
    root_walk_start(lds_mesh, lds_root, m, w);
    return LANE_WALK;
}
// The next mesh of a root-masked segment (mesh_done): false when none is left.
__device__ __forceinline__ bool next_root_mesh(const int2* lds_mesh, const float4* lds_root, int& mesh, MeshWalk& w) {
    const unsigned int rest = (unsigned int)mesh >> 8;
    if (!rest) return false;
    const int m = __builtin_ctz(rest);
    mesh = m | (int)((rest & (rest - 1u)) << 8);
    root_walk_start(lds_mesh, lds_root, m, w);
    return true;
}

// pixel_256_transform_gamma_corrected_kernel (:644-680) for one finished (pixel, pass) unit
// depth: the path's ray segments, counted into its band when the context measures band costs.
__device__ __forceinline__ void finish_unit(const DevTiling& til, const DevConfig& cfg, const DevOutput& out,
                                            const PathState& ps, unsigned int unit, int first_pass, int write_u8,
                                            int batch_log2, float clamp_hi, int depth) {
    if (til.band_cost) atomicAdd(&til.band_cost[pixel_band(til, unit_to_pixel(til, unit >> batch_log2))], (unsigned int)depth);
    const v3 c = clamp3(ps.rad, 0.0f, clamp_hi);
    if (batch_log2 == 0) {
        const int pixel = unit_to_pixel(til, unit);
        float* img = out.image + (size_t)pixel * 3;
        v3 sum;
        if (first_pass != 1) sum = mk3(img[0], img[1], img[2]) + c;
        else sum = c;
        img[0] = sum.x; img[1] = sum.y; img[2] = sum.z;
        if (write_u8 && out.image256) store_u8(cfg, sum, first_pass, out.image256 + (size_t)pixel * 3);
    } else {
        float* pr = out.pass_rad + (size_t)unit * 3;
        pr[0] = c.x; pr[1] = c.y; pr[2] = c.z;
    }
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---- the tail pool of pass_kernel_u -----------------------------------------------------------------
// Once a launch's work is drained, every wave runs until its last path ends, with fewer and fewer lanes
// busy: 18 % of the bench frame's walk steps come after the drain, with 8 of 64 lanes walking (PT_UPROF).
// So a drained wave other than wave 0 of its workgroup that holds at most donor_max paths hands each
// path that survives a shading batch to its part of a workgroup pool in LDS (the path state at a segment
// boundary: 64 B) and lets the lane go; such a wave ends early and its SIMD slot serves the next frame
// in flight. Wave 0 takes pooled paths into its free lanes and ends only when every other wave has
// ended and the pool is empty. A path continues exactly where it stopped (same state, same draws keyed
// by (pass, pixel, depth)), so results are unchanged. Slot protocol as pass_kernel_r: a FREE slot
// belongs to its donor wave, a FULL one to wave 0; data stores complete before the state store.
#define PT_TP_PART 32                               // pool slots per donor wave
#define PT_TP_SLOTS (PT_TP_PART * (PT_UBLOCK / 64 - 1))
template <int N>
__device__ __forceinline__ void tp_put(float4 (*q)[N], int s, const PathState& ps, unsigned int unit, int32_t pseed,
                                       int depth) {
    q[0][s] = make_float4(ps.o.x, ps.o.y, ps.o.z, ps.d.x);
    q[1][s] = make_float4(ps.d.y, ps.d.z, ps.thr.x, ps.thr.y);
    q[2][s] = make_float4(ps.thr.z, ps.rad.x, ps.rad.y, ps.rad.z);
    q[3][s] = make_float4(__uint_as_float(unit), __int_as_float(pseed), __int_as_float(ps.medium), __int_as_float(depth));
}
template <int N>
__device__ __forceinline__ void tp_get(float4 (*q)[N], int s, PathState& ps, unsigned int& unit, int32_t& pseed,
                                       int& depth) {
    const float4 a = q[0][s], b = q[1][s], c = q[2][s], e = q[3][s];
    ps.o = mk3(a.x, a.y, a.z);
    ps.d = mk3(a.w, b.x, b.y);
    ps.thr = mk3(b.z, b.w, c.x);
    ps.rad = mk3(c.y, c.z, c.w);
    unit = __float_as_uint(e.x); pseed = __float_as_int(e.y); ps.medium = __float_as_int(e.z); depth = __float_as_int(e.w);
}

// PROF: wave-level occupancy counters of the state machine into stats[16..23] (tools/uprof.py):
// rounds, walk steps, walking lanes summed over steps, shading batches, lanes shaded, triangle
// batches, lanes in triangle batches, lanes refilled.
// TP: the kernel has the tail pool (PT_TAIL_POOL > 0 selects it).
template <int MINW, bool PROF, bool QN, int CHAIN, bool PF, bool WIDE, int FEAT = PT_FEAT_ALL, bool TP = false>
__global__ __launch_bounds__(PT_UBLOCK, MINW) void pass_kernel_u(const LaunchParams* __restrict__ params, int first_pass,
                                                                int write_u8, int chunk, int batch_log2, int shade_min,
                                                                int walk_steps, int tri_min, int walk_min, int tail) {
    const int lane = threadIdx.x & 63;
    const LaunchParams* P0 = params;
    const float clamp_hi = (float)P0->cfg.max_depth * 2.0f;
    // workgroup copies in LDS: the first mesh ranges, every material and every sphere (the launch
    // reserves their bytes of dynamic LDS; pass_kernel_u runs only when that fits, PT_LDS_TABLES)
    __shared__ int2 lds_mesh[PT_LDS_MESHES];
    __shared__ int lds_wroot[WIDE ? PT_LDS_MESHES : 1];
    __shared__ int4 lds_next[PT_LDS_MESHES + 1];
    __shared__ float4 lds_root[2 * PT_ROOT_MESHES];
    __shared__ float4 tp_q[4][TP ? PT_TP_SLOTS : 1];
    __shared__ int tp_state[TP ? PT_TP_SLOTS : 1];        // 0 free, 1 full
    __shared__ int tp_scr[PT_UBLOCK / 64][TP ? PT_TP_SLOTS : 1];
    __shared__ int tp_donors;                    // waves other than wave 0 still running
    extern __shared__ float4 lds_dyn[];
    DevMaterial* lds_mats = reinterpret_cast<DevMaterial*>(lds_dyn);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int donor_max = TP ? (tail >> 16) & 0xff : 0;  // 0: no tail pool
    {
        const int2* mr = uniform_ptr(P0->sc.mesh_range);
        const int n = min(uniform_int(P0->sc.mesh_num), PT_LDS_MESHES);
        for (int i = threadIdx.x; i < n; i += PT_UBLOCK) lds_mesh[i] = mr[i];
        if (TP) {
            for (int i = threadIdx.x; i < PT_TP_SLOTS; i += PT_UBLOCK) tp_state[i] = 0;
            if (threadIdx.x == 0) tp_donors = PT_UBLOCK / 64 - 1;
        }
        if (WIDE) {
            const int* mw = uniform_ptr(P0->sc.mesh_wide);
            for (int i = threadIdx.x; i < n; i += PT_UBLOCK) lds_wroot[i] = mw[i];
        }
        const float4* ms = reinterpret_cast<const float4*>(uniform_ptr(P0->sc.materials));
        const int nm = uniform_int(P0->sc.material_num) * (int)(sizeof(DevMaterial) / 16);
        for (int i = threadIdx.x; i < nm; i += PT_UBLOCK) lds_dyn[i] = ms[i];
        const float4* sp = uniform_ptr(P0->sc.spheres);
        const int ns = uniform_int(P0->sc.sphere_num) * 2;
        for (int i = threadIdx.x; i < ns; i += PT_UBLOCK) lds_dyn[nm + i] = sp[i];
        __syncthreads();
        if (uniform_int(P0->sc.mesh_num) <= PT_LDS_MESHES) {  // lds_next (start_mesh_next)
            for (int i = threadIdx.x; i <= n; i += PT_UBLOCK) {
                int j = i;
                while (j < n && lds_mesh[j].x == lds_mesh[j].y) j++;
                lds_next[i] = j < n ? make_int4(lds_mesh[j].x, lds_mesh[j].y, j, 0) : make_int4(0, 0, n, 0);
            }
            if (!WIDE && PT_ROOT_SKIP && n <= PT_ROOT_MESHES) {  // lds_root (begin_segment_roots)
                const float4* nodes = uniform_ptr(P0->sc.nodes);
                for (int i = threadIdx.x; i < 2 * n; i += PT_UBLOCK) {
                    const int2 r = lds_mesh[i >> 1];
                    lds_root[i] = r.x != r.y ? nodes[2 * r.x + (i & 1)] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                }
            }
            __syncthreads();
        }
    }
    const float4* lds_spheres = lds_dyn + uniform_int(P0->sc.material_num) * (int)(sizeof(DevMaterial) / 16);

    PathState ps;
    v3 inv = mk3(0.0f, 0.0f, 0.0f);
    Hit h;
    MeshWalk w;
    int mesh = 0;
    int ptri = -1;  // leaf triangle awaiting its test (LANE_TRI)
    // DEF: deferred leaves (binary walk with prefetched triangles). dtri: the deferred leaf's triangle, -1
    // none, -2 the lane cannot defer (non-finite 1/d, or boxes not nested); de its box entry; pe the entry
    // of the leaf a lane is parked on (LANE_TRI; ptri -1: parked at its mesh's end behind a deferred leaf)
    constexpr bool DEF = PT_DEFER && CHAIN == 2 && PF && !QN && !WIDE;
    int dtri = -2;
    float de = 0.0f, pe = 0.0f;
    unsigned int unit = 0;
    int32_t pseed = 0;
    int depth = 0;
    int mode = LANE_WANT;
    unsigned long long segments = 0;  // wave-uniform: lanes shaded (ray segments traced)
    Counters none = {0u, 0u, 0u, 0u, 0u, 0u};
    const unsigned int units = (unsigned int)P0->til.unit_count << batch_log2;
    const EvenRegions regions{units, (units + PT_SHARDS - 1) / PT_SHARDS};
    WorkCursor cursor = work_begin();
    bool drained = false;
    unsigned long long prof[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tc = 0, tc2 = 0;
    // PROF timeline (stats[32..40]): this wave's start, the refill that first found the work drained,
    // its end (real-time clock), and the paths it shaded after the drain
    unsigned long long t_start = 0, t_drain = 0, tail_segments = 0;
    if (PROF) t_start = __builtin_amdgcn_s_memrealtime();
    while (true) {
        const LaunchParams* P = params;
        asm volatile("" : "+s"(P));
        P = uniform_ptr(P);
        DevScene sc = load_const(&P->sc);
        sc.materials = lds_mats;
        sc.spheres = lds_spheres;
        const DevConfig cfg = load_const(&P->cfg);
        const DevTiling til = load_const(&P->til);
        const DevOutput out = load_const(&P->out);
        const bool roots = !WIDE && !QN && PT_ROOT_SKIP && sc.mesh_num <= PT_ROOT_MESHES;  // wave-uniform
        if (PROF) { prof[0]++; tc = __builtin_readcyclecounter(); }

        // lanes without a path take the next (pixel, pass) units, one atomic per wave (pt_work.h)
        const bool want = mode == LANE_WANT;
        const unsigned long long need_mask = __ballot(want);
        if (need_mask) {
            const unsigned int u = work_take(out.fetch, regions.stride, regions, (unsigned int)chunk, need_mask, want,
                                             lanes_below(lane), cursor, drained);
            if (PROF) prof[7] += (unsigned long long)__popcll(__ballot(want && u != ~0u));
            if (PROF && drained && t_drain == 0) t_drain = __builtin_amdgcn_s_memrealtime();
            if (want) {
                if (u != ~0u) {
                    unit = u;
                    const int pixel = unit_to_pixel(til, u >> batch_log2);
                    const int32_t hseed = hash_pt(first_pass + (int)(u & ((1u << batch_log2) - 1u)));
                    const DevCamera cam = load_const(&P->cam);
                    if (PT_DUP == 4) {
                        PathState p2; int px2 = pixel, hs2 = hseed;
                        opaque(px2); opaque(hs2);
                        generate_path(cam, cfg, px2, hs2, &p2);
                        opaque(p2);
                    }
                    generate_path(cam, cfg, pixel, hseed, &ps);
                    pseed = path_seed(hseed, pixel);
                    depth = 0;
                    if (cfg.max_depth > 0) {
                        mode = LANE_NEW;
                    } else {
                        finish_unit(til, cfg, out, ps, unit, first_pass, write_u8, batch_log2, clamp_hi, depth);
                    }
                } else if (drained) {
                    mode = LANE_DONE;
                }
            }
        }
        if (TP && donor_max && drained && wid != 0) {
            // a drained wave with few paths left hands its survivors to the pool (tail pool above)
            const unsigned long long surv = __ballot(mode == LANE_NEW);
            const int live = __popcll(__ballot(mode != LANE_DONE && mode != LANE_WANT));
            if (surv && live <= donor_max) {
                volatile int* tst = tp_state;
                int* scr = tp_scr[wid];
                const unsigned long long below = lanes_below(lane);
                const int base = (wid - 1) * PT_TP_PART;
                const int sv = lane < PT_TP_PART ? tst[base + lane] : 1;
                const unsigned long long fr = __ballot(sv == 0);
                if (sv == 0) scr[__popcll(fr & below)] = base + lane;
                lds_fence();
                const int r = __popcll(surv & below);
                int slot = -1;
                if (mode == LANE_NEW && r < __popcll(fr)) {
                    slot = scr[r];
                    tp_put(tp_q, slot, ps, unit, pseed, depth);
                    mode = LANE_DONE;
                }
                lds_fence();
                if (slot >= 0) tst[slot] = 1;
            }
        }
        if (TP && donor_max && wid == 0 && drained) {
            // wave 0 takes pooled paths into its free lanes (see the tail pool above); with no path in
            // any lane it waits here until the pool has one or every other wave has ended
            const unsigned long long freem = __ballot(mode == LANE_DONE);
            if (freem) {
                volatile int* tst = tp_state;
                int v0, v1, n0, nfull;
                unsigned long long f0, f1;
                while (true) {
                    const int donors_left = *(volatile int*)&tp_donors;
                    lds_fence();  // the pool is scanned after the count is read
                    v0 = lane < PT_TP_SLOTS ? tst[lane] : 0;
                    v1 = lane + 64 < PT_TP_SLOTS ? tst[lane + 64] : 0;
                    f0 = __ballot(v0 == 1);
                    f1 = __ballot(v1 == 1);
                    n0 = __popcll(f0);
                    nfull = n0 + __popcll(f1);
                    if (nfull || donors_left == 0 || freem != ~0ull) break;
                    __builtin_amdgcn_s_sleep(2);
                }
                if (nfull) {
                    int* scr = tp_scr[0];
                    const unsigned long long below = lanes_below(lane);
                    if (v0 == 1) scr[__popcll(f0 & below)] = lane;
                    if (v1 == 1) scr[n0 + __popcll(f1 & below)] = lane + 64;
                    lds_fence();
                    const int k = __popcll(freem & below);
                    int slot = -1;
                    if (mode == LANE_DONE && k < nfull) {
                        slot = scr[k];
                        tp_get(tp_q, slot, ps, unit, pseed, depth);
                        mode = LANE_NEW;
                    }
                    lds_fence();
                    if (slot >= 0) tst[slot] = 0;
                }
            }
        }
        if (mode == LANE_NEW) {
            if (roots) mode = begin_segment_roots(sc, lds_mesh, lds_root, ps, inv, h, w, mesh);
            else mode = begin_segment<WIDE>(sc, lds_mesh, ps, inv, h, w, mesh);
            if (DEF)
                dtri = sc.nested && __builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z)
                           ? -1 : -2;
        }
        if (!__any(mode != LANE_DONE)) break;
        if (PROF) { const unsigned long long t = __builtin_readcyclecounter(); prof[8] += t - tc; tc = t; }

        const unsigned long long ready = __ballot(mode == LANE_READY);
        const unsigned long long walking = __ballot(mode == LANE_WALK || mode == LANE_TRI);
        // once the launch's work is drained (wave-uniform) the wave only finishes its paths: its
        // thresholds switch to the tail pair (tail = shade_min | walk_min << 8)
        const unsigned int smin = drained ? (unsigned int)(tail & 0xff) : (unsigned int)shade_min;
        const unsigned int wmin = drained ? (unsigned int)(tail >> 8) : (unsigned int)walk_min;
        if (ready && (__popcll(walking) <= wmin || __popcll(ready) >= smin)) {
            if (PROF) { prof[3]++; prof[4] += (unsigned long long)__popcll(ready); }
            if (PROF && drained) tail_segments += (unsigned long long)__popcll(ready);
            segments += (unsigned long long)__popcll(ready);
            bool alive = false;
            if (mode == LANE_READY) {
                // the rest of trace_ray_kernel for this segment (:456-624)
                if (PT_DUP == 1) {
                    PathState p2 = ps; Hit h2 = h; int d2 = depth;
                    opaque(p2); opaque(h2); opaque(d2);
                    bool a2 = shade_hit<false, FEAT>(sc, cfg, d2, pseed, &p2, h2, &none, nullptr);
                    opaque(p2); opaque(a2);
                }
                alive = shade_hit<false, FEAT>(sc, cfg, depth, pseed, &ps, h, &none, nullptr);
            }
            if (PROF) tc2 = __builtin_readcyclecounter();
            if (mode == LANE_READY) {  // the pass's end for this unit, or the next trace step
                depth++;
                if (!alive || depth >= cfg.max_depth) {
                    finish_unit(til, cfg, out, ps, unit, first_pass, write_u8, batch_log2, clamp_hi, depth);
                    mode = LANE_WANT;
                } else {
                    mode = LANE_NEW;  // its next segment starts in the next round's refill, with the new paths
                }
            }
            if (PROF) prof[15] += __builtin_readcyclecounter() - tc2;
            if (PROF) prof[9] += __builtin_readcyclecounter() - tc;
            continue;
        }

        const __amdgpu_buffer_rsrc_t rn = make_rsrc(sc.nodes, sc.node_count * 32);
        const __amdgpu_buffer_rsrc_t rt = make_rsrc(sc.tri_geom, sc.tri_count * 48);
        const __amdgpu_buffer_rsrc_t rw = WIDE ? make_rsrc(sc.wide, sc.wide_count * 128) : rn;
        __amdgpu_buffer_rsrc_t rq = rn;
        float4 fb = make_float4(0.0f, 0.0f, 0.0f, 0.0f), fs = fb;
        if (QN) {
            rq = make_rsrc(sc.qnodes, sc.node_count * 16);
            fb = load_const(sc.mesh_q);
            fs = load_const(sc.mesh_q + 1);
        }
        // closest_hit's merge of a finished mesh walk (:443-454), then the next mesh or READY
        auto mesh_done = [&]() {
            if (w.tri >= 0 && w.t < h.t) {
                h.t = w.t; h.t1 = w.t1; h.t2 = w.t2; h.prim = w.tri; h.type = 2;
            }
            bool more;
            if (roots) {
                more = next_root_mesh(lds_mesh, lds_root, mesh, w);
            } else {
                mesh++;
                if (PT_NEXT_MESH && !WIDE && sc.mesh_num <= PT_LDS_MESHES) more = start_mesh_next(lds_next, mesh, w);
                else more = start_mesh(sc, lds_mesh, lds_wroot, WIDE && w.end < 0, mesh, w);
            }
            mode = more ? LANE_WALK : LANE_READY;
        };
        // PF: the parked triangle's geometry, loaded at the park; scoped to the walk loop, which no lane
        // leaves parked (the last step flushes the batch), so it is not live across shading
        float4 pta = make_float4(0.0f, 0.0f, 0.0f, 0.0f), ptb = pta, ptc = pta;
        constexpr bool KEEP = PT_KEEP_PARKED && PF && !QN && !DEF;
        if (KEEP && mode == LANE_TRI) {  // parked in an earlier round: its triangle's loads again
            pta = bload(rt, ptri * 48); ptb = bload(rt, ptri * 48 + 16); ptc = bload(rt, ptri * 48 + 32);
        }
        for (int k = 0; k < walk_steps; k++) {
            if (k > 0 && !__any(mode == LANE_WALK || mode == LANE_TRI)) break;
            if (PROF) {
                prof[1]++; prof[2] += (unsigned long long)__popcll(__ballot(mode == LANE_WALK));
                prof[12] += (unsigned long long)__popcll(__ballot(mode == LANE_TRI));
#if PT_PROF_MESH  // diagnostic builds: walking lanes per mesh (meshes 0, 1, 2) instead of the drained/ready/idle counts
                prof[11] += (unsigned long long)__popcll(__ballot(mode == LANE_WALK && (mesh & 0xff) == 0));
                prof[13] += (unsigned long long)__popcll(__ballot(mode == LANE_WALK && (mesh & 0xff) == 1));
                prof[14] += (unsigned long long)__popcll(__ballot(mode == LANE_WALK && (mesh & 0xff) == 2));
#else
                if (drained) prof[11] += 1ull | ((unsigned long long)__popcll(__ballot(mode == LANE_WALK)) << 32);
                prof[13] += (unsigned long long)__popcll(__ballot(mode == LANE_READY));
                prof[14] += (unsigned long long)__popcll(__ballot(mode == LANE_WANT || mode == LANE_DONE));
#endif
            }
            if (mode == LANE_WALK) {
                if (PT_DUP == 2) {
                    MeshWalk w2 = w; v3 o2 = ps.o, i2 = inv; int t2 = ptri;
                    opaque(w2); opaque(o2); opaque(i2);
                    bool l2 = walk_box(rn, o2, i2, w2, t2);
                    opaque(w2); opaque(l2); opaque(t2);
                }
                bool leaf;
                float le = 0.0f;
                if (WIDE && w.end < 0) leaf = walk_wide(rw, ps.o, inv, w, ptri);
                else leaf = QN ? walk_box_q(rq, fb, fs, ps.o, inv, w, ptri)
                               : (CHAIN > 1 ? walk_box_chain<CHAIN>(rn, ps.o, inv, w, ptri, le) : walk_box(rn, ps.o, inv, w, ptri));
                if (DEF) {
                    // a lane without a deferred leaf defers this one: it walks on past it, the triangle's loads
                    // in flight until its batch; with one deferred already (or unable to defer) it parks.
                    // Selects rather than branches: the exec-mask bookkeeping of a branchy form costs more
                    // scalar issue than the batching saves
                    const bool defer = leaf && dtri == -1;
                    if (leaf && dtri < 0) {
                        pta = bload(rt, ptri * 48); ptb = bload(rt, ptri * 48 + 16); ptc = bload(rt, ptri * 48 + 32);
                    }
                    dtri = defer ? ptri : dtri;
                    de = defer ? le : de;
                    pe = le;
                    w.pos += defer ? 1 : 0;
                    mode = leaf && !defer ? LANE_TRI : mode;
                } else if (leaf) {
                    mode = LANE_TRI;
                    pe = le;
                    if (PF && !QN && (!DEF || dtri < 0)) {  // the triangle's loads are in flight while the batch fills
                        pta = bload(rt, ptri * 48); ptb = bload(rt, ptri * 48 + 16); ptc = bload(rt, ptri * 48 + 32);
                    }
                } else if (!PT_MESH_SITE && w.pos == w.end) {
                    mesh_done();
                }
            }
            // leaf triangles are tested in batches of at least tri_min lanes (or when no lane can
            // walk on): the triangle test then runs with many lanes active instead of one or two
            const bool in_batch = mode == LANE_TRI || (DEF && dtri >= 0);
            const unsigned long long pend = __ballot(in_batch);
            // PF: no lane leaves the walk loop parked, so the prefetched geometry never lives across shading
            if (pend && (__popcll(pend) >= (unsigned int)tri_min || !__any(mode == LANE_WALK) ||
                         (PF && !KEEP && k == walk_steps - 1))) {
                if (PROF) { prof[5]++; prof[6] += (unsigned long long)__popcll(pend); }
                if (DEF) {
                    if (in_batch) {
                        // the earliest unresolved leaf: the deferred one, else the one the lane is parked on;
                        // it counts if its box still passes under the min_t its preorder position sees
                        const bool d = dtri >= 0;
                        walk_tri_geom_if(pta, ptb, ptc, ps.o, ps.d, w, d ? dtri : ptri, (d ? de : pe) <= w.t);
                        // a second leaf parked behind the deferred one becomes the deferred leaf if its box
                        // still passes (a leaf's skip index is the next record: pos + 1 either way); a lane
                        // parked at its mesh's end (ptri -1) stays there for mesh_done
                        const bool parked = mode == LANE_TRI;
                        const int nt = parked && d && ptri >= 0 && pe <= w.t ? ptri : -1;
                        w.pos += parked && (!d || ptri >= 0) ? 1 : 0;
                        mode = parked ? LANE_WALK : mode;
                        dtri = d ? nt : dtri;
                        de = pe;
                        if (nt >= 0) {
                            pta = bload(rt, nt * 48); ptb = bload(rt, nt * 48 + 16); ptc = bload(rt, nt * 48 + 32);
                        }
                    }
                    // the round's last step: no lane leaves the walk loop with a deferred leaf
                    if (k == walk_steps - 1 && dtri >= 0) {
                        walk_tri_geom_if(pta, ptb, ptc, ps.o, ps.d, w, dtri, de <= w.t);
                        dtri = -1;
                    }
                } else if (mode == LANE_TRI) {
                    if (QN) walk_tri_q(rn, rt, ps.o, ps.d, inv, w, ptri);
                    else {
                        if (PT_DUP == 3) {
                            MeshWalk w2 = w; v3 o2 = ps.o, d2 = ps.d; int t2 = ptri;
                            opaque(w2); opaque(o2); opaque(d2); opaque(t2);
                            walk_tri(rt, o2, d2, w2, t2);
                            opaque(w2);
                        }
                        const bool advance = !(WIDE && w.end < 0);  // walk_wide already moved past the leaf
                        if (PF) walk_tri_geom(pta, ptb, ptc, ps.o, ps.d, w, ptri, advance);
                        else walk_tri(rt, ps.o, ps.d, w, ptri, advance);
                    }
                    mode = LANE_WALK;
                    if (!PT_MESH_SITE && w.pos == w.end) mesh_done();
                }
            }
            // a lane whose mesh walk ended in this step (after a box or after its triangle) merges it and
            // starts the next mesh: one mesh_done site for both (PT_MESH_SITE=0 builds: two); with a leaf
            // still deferred it parks until that leaf is resolved
            if (DEF) {
                const bool at_end = mode == LANE_WALK && w.pos == w.end;
                const bool wait = at_end && dtri >= 0;
                mode = wait ? LANE_TRI : mode;
                ptri = wait ? -1 : ptri;
                if (at_end && !wait) mesh_done();
            } else if (PT_MESH_SITE && mode == LANE_WALK && w.pos == w.end) {
                mesh_done();
            }
        }
        if (PROF) prof[10] += __builtin_readcyclecounter() - tc;
    }

    if (TP && donor_max && wid != 0 && lane == 0) {
        lds_fence();  // this wave's pool stores before its exit is counted
        atomicSub(&tp_donors, 1);
    }
    if (lane == 0) {
        atomicAdd(&P0->out.stats[0], segments);
        if (PROF) {
#pragma unroll
            for (int k = 0; k < 16; k++) atomicAdd(&P0->out.stats[16 + k], prof[k]);
            // minima as maxima of the complement, so a zeroed buffer starts every slot
            const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
            if (t_drain == 0) t_drain = t_end;
            unsigned long long* tl = P0->out.stats + 32;
            atomicMax(&tl[0], ~t_start); atomicMax(&tl[1], t_start);
            atomicMax(&tl[2], ~t_drain); atomicMax(&tl[3], t_drain);
            atomicMax(&tl[4], ~t_end); atomicMax(&tl[5], t_end);
            atomicAdd(&tl[6], t_end - t_drain); atomicAdd(&tl[7], t_end - t_start);
            atomicAdd(&tl[8], 1ull); atomicAdd(&tl[9], tail_segments);
        }
    }
}

// ---- pass_kernel_r: walker waves and shader waves regrouping paths through LDS ------------------
// In pass_kernel_u every wave both walks and shades, so a wave shades whatever subset of its lanes is
// ready (about 40 of 64 on the bench frame) and walks with the lanes that are not. Here a workgroup's
// waves take fixed roles. NWALK walker waves only walk: a lane whose closest hit is known hands its
// path (state and hit) to a slot of its wave's partition of PT_RG_PART LDS slots and takes a path
// that waits there for its next segment (a swap through one slot), or a new (pixel, pass) unit.
// NSHADE shader waves only shade: shader k serves the slots s with s % NSHADE == k, takes up to 64
// waiting paths at a time (shade_min of them, or fewer once it has waited rg_spin rounds), runs
// shade_hit on them, and writes a surviving path back into its slot for the walkers, or finishes
// the unit. Every path still computes exactly the reference sequence: the same walk, the same shade,
// the same draws keyed by (pass, pixel, depth); only the lane that runs each step changes.
//
// Slot ownership makes the exchange lock-free: a FREE or WALK slot belongs to its walker wave, a
// SHADE slot to its shader wave, and only the owner moves a slot to the next state, after its data
// stores have completed (s_waitcnt lgkmcnt(0) between the data and the state store; readers load the
// state first). A walker wave exits once the work is drained, none of its lanes holds a path and its
// partition is all FREE; the shader waves exit once every walker wave has exited.
#define PT_RG_PART 64
#define PT_RG_IDLE_CAP (1 << 24)  // idle rounds after which a wave gives up (never reached by a correct run)
enum : int { SLOT_FREE = 0, SLOT_WALK = 1, SLOT_SHADE = 2 };


// q0 (o, d.x) q1 (d.y, d.z, thr.x, thr.y) q2 (thr.z, rad) q3 (unit, pseed, medium, depth) q4 (hit)
__device__ __forceinline__ void slot_put(float4* const q[5], int s, const PathState& ps, unsigned int unit, int32_t pseed,
                                         int depth, const Hit* h) {
    q[0][s] = make_float4(ps.o.x, ps.o.y, ps.o.z, ps.d.x);
    q[1][s] = make_float4(ps.d.y, ps.d.z, ps.thr.x, ps.thr.y);
    q[2][s] = make_float4(ps.thr.z, ps.rad.x, ps.rad.y, ps.rad.z);
    q[3][s] = make_float4(__uint_as_float(unit), __int_as_float(pseed), __int_as_float(ps.medium), __int_as_float(depth));
    if (h) q[4][s] = make_float4(h->t, h->t1, h->t2, __int_as_float(h->prim * 4 + h->type));
}

__device__ __forceinline__ void slot_get(float4* const q[5], int s, PathState& ps, unsigned int& unit, int32_t& pseed,
                                         int& depth, Hit* h) {
    const float4 a = q[0][s], b = q[1][s], c = q[2][s], e = q[3][s];
    ps.o = mk3(a.x, a.y, a.z);
    ps.d = mk3(a.w, b.x, b.y);
    ps.thr = mk3(b.z, b.w, c.x);
    ps.rad = mk3(c.y, c.z, c.w);
    unit = __float_as_uint(e.x); pseed = __float_as_int(e.y); ps.medium = __float_as_int(e.z); depth = __float_as_int(e.w);
    if (h) {
        const float4 f = q[4][s];
        const int pt = __float_as_int(f.w);
        h->t = f.x; h->t1 = f.y; h->t2 = f.z; h->type = pt & 3; h->prim = pt >> 2;
    }
}

// PROF counters (stats[16..], tools/rgprof.py): walker rounds, handoffs, lanes handed to shading, walk
// steps, walking lanes summed over steps, walker idle rounds, shader batches, lanes shaded, shader idle
// rounds, triangle batches, then cycles: walker handoff, walker walk, walker idle, shader shading,
// shader idle, lanes in triangle batches.
template <int MINW, int NWALK, int NSHADE, bool PROF, int FEAT>
__global__ __launch_bounds__((NWALK + NSHADE) * 64, MINW) void pass_kernel_r(
    const LaunchParams* __restrict__ params, int first_pass, int write_u8, int chunk, int batch_log2, int shade_min,
    int walk_steps, int tri_min, int walk_min, int rg) {
    constexpr int NT = (NWALK + NSHADE) * 64;
    constexpr int S = NWALK * PT_RG_PART;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LaunchParams* P0 = params;
    const float clamp_hi = (float)P0->cfg.max_depth * 2.0f;
    const unsigned long long below = lanes_below(lane);
    __shared__ int2 lds_mesh[PT_LDS_MESHES];
    __shared__ int4 lds_next[PT_LDS_MESHES + 1];
    __shared__ float4 slot_q[5][S];
    __shared__ int slot_state[S];
    __shared__ int scratch[NWALK + NSHADE][128];
    __shared__ int walkers_done;
    extern __shared__ float4 lds_dyn[];
    DevMaterial* lds_mats = reinterpret_cast<DevMaterial*>(lds_dyn);
    {
        const int2* mr = uniform_ptr(P0->sc.mesh_range);
        const int n = min(uniform_int(P0->sc.mesh_num), PT_LDS_MESHES);
        for (int i = threadIdx.x; i < n; i += NT) lds_mesh[i] = mr[i];
        const float4* ms = reinterpret_cast<const float4*>(uniform_ptr(P0->sc.materials));
        const int nm = uniform_int(P0->sc.material_num) * (int)(sizeof(DevMaterial) / 16);
        for (int i = threadIdx.x; i < nm; i += NT) lds_dyn[i] = ms[i];
        const float4* sp = uniform_ptr(P0->sc.spheres);
        const int ns = uniform_int(P0->sc.sphere_num) * 2;
        for (int i = threadIdx.x; i < ns; i += NT) lds_dyn[nm + i] = sp[i];
        for (int i = threadIdx.x; i < S; i += NT) slot_state[i] = SLOT_FREE;
        if (threadIdx.x == 0) walkers_done = 0;
        __syncthreads();
        if (uniform_int(P0->sc.mesh_num) <= PT_LDS_MESHES) {  // lds_next (start_mesh_next)
            for (int i = threadIdx.x; i <= n; i += NT) {
                int j = i;
                while (j < n && lds_mesh[j].x == lds_mesh[j].y) j++;
                lds_next[i] = j < n ? make_int4(lds_mesh[j].x, lds_mesh[j].y, j, 0) : make_int4(0, 0, n, 0);
            }
            __syncthreads();
        }
    }
    const float4* lds_spheres = lds_dyn + uniform_int(P0->sc.material_num) * (int)(sizeof(DevMaterial) / 16);
    float4* const q[5] = {slot_q[0], slot_q[1], slot_q[2], slot_q[3], slot_q[4]};
    volatile int* st = slot_state;
    int* scr = scratch[wid];
    unsigned long long prof[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long segments = 0;
    int idle = 0;
    bool capped = false;
    unsigned long long tc = 0;

    if (wid < NWALK) {
        // ---------------- walker wave ----------------
        const int pbase = wid * PT_RG_PART;
        PathState ps;
        v3 inv = mk3(0.0f, 0.0f, 0.0f);
        Hit h;
        MeshWalk w;
        int mesh = 0;
        int ptri = -1;
        unsigned int unit = 0;
        int32_t pseed = 0;
        int depth = 0;
        int mode = LANE_WANT;
        const unsigned int units = (unsigned int)P0->til.unit_count << batch_log2;
        const EvenRegions regions{units, (units + PT_SHARDS - 1) / PT_SHARDS};
        WorkCursor cursor = work_begin();
        bool drained = false;
        while (true) {
            const LaunchParams* P = params;
            asm volatile("" : "+s"(P));
            P = uniform_ptr(P);
            DevScene sc = load_const(&P->sc);
            sc.materials = lds_mats;
            sc.spheres = lds_spheres;
            const DevConfig cfg = load_const(&P->cfg);
            const DevTiling til = load_const(&P->til);
            const DevOutput out = load_const(&P->out);
            if (PROF) { prof[0]++; tc = __builtin_readcyclecounter(); }
            const unsigned long long ready = __ballot(mode == LANE_READY);
            const unsigned long long wantm = __ballot(mode == LANE_WANT);
            const unsigned int nwalking = (unsigned int)__popcll(__ballot(mode == LANE_WALK || mode == LANE_TRI));
            if ((ready | wantm) && (__popcll(ready) >= shade_min || nwalking <= (unsigned int)walk_min)) {
                if (PROF) prof[1]++;
                // the partition's slots: WALK ones hold paths waiting for their next segment
                const int sv = st[pbase + lane];
                const unsigned long long wq = __ballot(sv == SLOT_WALK), fr = __ballot(sv == SLOT_FREE);
                if (sv == SLOT_WALK) scr[__popcll(wq & below)] = pbase + lane;
                if (sv == SLOT_FREE) scr[64 + __popcll(fr & below)] = pbase + lane;
                lds_fence();
                const int nwq = __popcll(wq), nfr = __popcll(fr);
                const int nrdy = __popcll(ready);
                if (drained && nwalking == 0 && !ready && wantm == ~0ull && fr == ~0ull) break;
                // ready lanes hand their path over: swap with a waiting path, else into a free slot
                int mark = -1;
                if (mode == LANE_READY) {
                    const int r = __popcll(ready & below);
                    if (r < nwq) {
                        mark = scr[r];
                        PathState np; unsigned int nu; int32_t nseed; int nd;
                        slot_get(q, mark, np, nu, nseed, nd, nullptr);
                        slot_put(q, mark, ps, unit, pseed, depth, &h);
                        ps = np; unit = nu; pseed = nseed; depth = nd;
                        mode = LANE_NEW;
                    } else if (r - nwq < nfr) {
                        mark = scr[64 + r - nwq];
                        slot_put(q, mark, ps, unit, pseed, depth, &h);
                        mode = LANE_WANT;
                    }
                }
                if (PROF) prof[2] += (unsigned long long)__popcll(__ballot(mark >= 0));
                lds_fence();
                if (mark >= 0) st[mark] = SLOT_SHADE;
                // lanes without a path take the remaining waiting paths
                const int nswap = nrdy < nwq ? nrdy : nwq;
                const unsigned long long want2 = __ballot(mode == LANE_WANT);
                int pulled = -1;
                if (mode == LANE_WANT) {
                    const int k = nswap + __popcll(want2 & below);
                    if (k < nwq) {
                        pulled = scr[k];
                        slot_get(q, pulled, ps, unit, pseed, depth, nullptr);
                        mode = LANE_NEW;
                    }
                }
                lds_fence();
                if (pulled >= 0) st[pulled] = SLOT_FREE;
                // and then new (pixel, pass) units (pt_work.h)
                const bool want = mode == LANE_WANT;
                const unsigned long long need_mask = __ballot(want);
                if (need_mask && !drained) {
                    const unsigned int u = work_take(out.fetch, regions.stride, regions, (unsigned int)chunk, need_mask,
                                                     want, below, cursor, drained);
                    if (want && u != ~0u) {
                        unit = u;
                        const int pixel = unit_to_pixel(til, u >> batch_log2);
                        const int32_t hseed = hash_pt(first_pass + (int)(u & ((1u << batch_log2) - 1u)));
                        const DevCamera cam = load_const(&P->cam);
                        generate_path(cam, cfg, pixel, hseed, &ps);
                        pseed = path_seed(hseed, pixel);
                        depth = 0;
                        if (cfg.max_depth > 0) mode = LANE_NEW;
                        else finish_unit(til, cfg, out, ps, unit, first_pass, write_u8, batch_log2, clamp_hi, depth);
                    }
                }
                if (mode == LANE_NEW) mode = begin_segment<false>(sc, lds_mesh, ps, inv, h, w, mesh);
                if (!__any(mode == LANE_WALK || mode == LANE_TRI)) {  // waiting for the shader waves
                    if (PROF) prof[5]++;
                    if (++idle > PT_RG_IDLE_CAP) { capped = true; break; }
                    __builtin_amdgcn_s_sleep(2);
                    if (PROF) prof[12] += __builtin_readcyclecounter() - tc;
                    continue;
                }
                idle = 0;
            }
            if (PROF) { const unsigned long long t = __builtin_readcyclecounter(); prof[10] += t - tc; tc = t; }

            const __amdgpu_buffer_rsrc_t rn = make_rsrc(sc.nodes, sc.node_count * 32);
            const __amdgpu_buffer_rsrc_t rt = make_rsrc(sc.tri_geom, sc.tri_count * 48);
            auto mesh_done = [&]() {
                if (w.tri >= 0 && w.t < h.t) {
                    h.t = w.t; h.t1 = w.t1; h.t2 = w.t2; h.prim = w.tri; h.type = 2;
                }
                mesh++;
                const bool more = sc.mesh_num <= PT_LDS_MESHES ? start_mesh_next(lds_next, mesh, w)
                                                               : start_mesh(sc, lds_mesh, nullptr, false, mesh, w);
                mode = more ? LANE_WALK : LANE_READY;
            };
            float4 pta = make_float4(0.0f, 0.0f, 0.0f, 0.0f), ptb = pta, ptc = pta;
            for (int k = 0; k < walk_steps; k++) {
                if (k > 0 && !__any(mode == LANE_WALK || mode == LANE_TRI)) break;
                if (PROF) { prof[3]++; prof[4] += (unsigned long long)__popcll(__ballot(mode == LANE_WALK)); }
                if (mode == LANE_WALK) {
                    const bool leaf = walk_box_chain<2>(rn, ps.o, inv, w, ptri);
                    if (leaf) {
                        mode = LANE_TRI;
                        pta = bload(rt, ptri * 48); ptb = bload(rt, ptri * 48 + 16); ptc = bload(rt, ptri * 48 + 32);
                    } else if (w.pos == w.end) {
                        mesh_done();
                    }
                }
                const unsigned long long pend = __ballot(mode == LANE_TRI);
                if (pend && (__popcll(pend) >= (unsigned int)tri_min || !__any(mode == LANE_WALK) || k == walk_steps - 1)) {
                    if (PROF) { prof[9]++; prof[15] += (unsigned long long)__popcll(pend); }
                    if (mode == LANE_TRI) {
                        walk_tri_geom(pta, ptb, ptc, ps.o, ps.d, w, ptri, true);
                        mode = LANE_WALK;
                        if (w.pos == w.end) mesh_done();
                    }
                }
            }
            if (PROF) prof[11] += __builtin_readcyclecounter() - tc;
        }
        if (lane == 0) atomicAdd(&walkers_done, 1);
    } else {
        // ---------------- shader wave ----------------
        const int k = wid - NWALK;
        constexpr int NS = (S + NSHADE - 1) / NSHADE;  // slots served (k + NSHADE * j, j < NS)
        constexpr int NC = (NS + 63) / 64;
        const int spin_max = rg & 0xffff;
        const int batch_min = rg >> 16;
        int spins = 0;
        int start = 0;  // first chunk scanned: rotates so that no partition waits behind the others
        while (true) {
            const LaunchParams* P = params;
            asm volatile("" : "+s"(P));
            P = uniform_ptr(P);
            DevScene sc = load_const(&P->sc);
            sc.materials = lds_mats;
            sc.spheres = lds_spheres;
            const DevConfig cfg = load_const(&P->cfg);
            const DevTiling til = load_const(&P->til);
            const DevOutput out = load_const(&P->out);
            if (PROF) tc = __builtin_readcyclecounter();
            unsigned long long m[NC];
            int total = 0;
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const int j = c * 64 + lane;
                const int s = k + NSHADE * j;
                const int sv = (j < NS && s < S) ? st[s] : SLOT_FREE;
                m[c] = __ballot(sv == SLOT_SHADE);
                total += __popcll(m[c]);
            }
            if (total == 0 || (total < batch_min && spins < spin_max)) {
                if (total == 0 && *(volatile int*)&walkers_done == NWALK) break;
                spins++;
                if (PROF) prof[8]++;
                if (++idle > PT_RG_IDLE_CAP) { capped = true; break; }
                __builtin_amdgcn_s_sleep(1);
                if (PROF) prof[14] += __builtin_readcyclecounter() - tc;
                continue;
            }
            spins = 0;
            idle = 0;
            // the first 64 waiting paths, from chunk `start` on: lane r takes the r-th
            int base = 0;
#pragma unroll
            for (int cc = 0; cc < NC; cc++) {
                const int c = (start + cc) % NC;
                const int r = base + __popcll(m[c] & below);
                if (((m[c] >> lane) & 1ull) && r < 64) scr[r] = k + NSHADE * (c * 64 + lane);
                base += __popcll(m[c]);
            }
            start = (start + 1) % NC;
            lds_fence();
            const int n = total < 64 ? total : 64;
            const bool have = lane < n;
            int s = -1;
            PathState ps;
            Hit h;
            unsigned int unit = 0;
            int32_t pseed = 0;
            int depth = 0;
            bool alive = false;
            if (have) {
                s = scr[lane];
                slot_get(q, s, ps, unit, pseed, depth, &h);
                Counters none = {0u, 0u, 0u, 0u, 0u, 0u};
                alive = shade_hit<false, FEAT>(sc, cfg, depth, pseed, &ps, h, &none);
                depth++;
            }
            segments += (unsigned long long)n;
            if (PROF) { prof[6]++; prof[7] += (unsigned long long)n; }
            int next = SLOT_FREE;
            if (have) {
                if (!alive || depth >= cfg.max_depth) {
                    finish_unit(til, cfg, out, ps, unit, first_pass, write_u8, batch_log2, clamp_hi, depth);
                } else {
                    slot_put(q, s, ps, unit, pseed, depth, nullptr);
                    next = SLOT_WALK;
                }
            }
            lds_fence();
            if (have) st[s] = next;
            if (PROF) prof[13] += __builtin_readcyclecounter() - tc;
        }
    }

    if (lane == 0) {
        atomicAdd(&P0->out.stats[0], segments);
        if (capped) atomicAdd(&P0->out.stats[PT_STAT_RG_CAPPED], 1ull);  // checked by the host after the frame
        if (PROF) {
#pragma unroll
            for (int i = 0; i < 16; i++) atomicAdd(&P0->out.stats[16 + i], prof[i]);
        }
    }
}

// The running sum over a batch of passes, in pass order (path_tracer_kernel.cu:644-651 applied
// pass after pass), then the 8-bit output of the batch's last pass.
__global__ __launch_bounds__(PT_BLOCK) void accumulate_kernel(const LaunchParams* __restrict__ P, int first_pass,
                                                              int batch_log2, int write_u8) {
    const unsigned int lu = blockIdx.x * PT_BLOCK + threadIdx.x;
    if (lu >= (unsigned int)P->til.unit_count) return;
    const int pixel = unit_to_pixel(P->til, lu);
    const int batch = 1 << batch_log2;
    float* img = P->out.image + (size_t)pixel * 3;
    const float* pr = P->out.pass_rad + ((size_t)lu << batch_log2) * 3;
    v3 sum = first_pass == 1 ? mk3(0.0f, 0.0f, 0.0f) : mk3(img[0], img[1], img[2]);  // pass 1 overwrites
    if ((batch & 3) == 0) {  // four passes = 12 floats = three 16-B loads (the unit's run is 16-B aligned)
        const float4* q = reinterpret_cast<const float4*>(pr);
        for (int g = 0; g < batch / 4; g++) {
            const float4 a = q[3 * g], b = q[3 * g + 1], c = q[3 * g + 2];
            const v3 cs[4] = {mk3(a.x, a.y, a.z), mk3(a.w, b.x, b.y), mk3(b.z, b.w, c.x), mk3(c.y, c.z, c.w)};
#pragma unroll
            for (int t = 0; t < 4; t++) sum = (first_pass + 4 * g + t == 1) ? cs[t] : sum + cs[t];
        }
    } else {
        for (int j = 0; j < batch; j++) {
            const v3 c = mk3(pr[3 * j], pr[3 * j + 1], pr[3 * j + 2]);
            sum = (first_pass + j == 1) ? c : sum + c;
        }
    }
    img[0] = sum.x; img[1] = sum.y; img[2] = sum.z;
    if (write_u8 && P->out.image256)
        store_u8(P->cfg, sum, first_pass + batch - 1, P->out.image256 + (size_t)pixel * 3);
}

// Gamma/8-bit from a float running sum (used after a multi-GPU reduce, and by the reference
// ABI when the caller asks for the 8-bit image only at the end of a frame).
__global__ __launch_bounds__(PT_BLOCK) void u8_kernel(DevConfig cfg, const float* image, uint8_t* image256,
                                                      int pixel_count, int pass) {
    int i = blockIdx.x * PT_BLOCK + threadIdx.x;
    if (i >= pixel_count) return;
    const float* p = image + (size_t)i * 3;
    store_u8(cfg, mk3(p[0], p[1], p[2]), pass, image256 + (size_t)i * 3);
}

// Per-material constants of shade_hit (DevMaterial::rough_alpha / tir_front / tir_back), with the
// expressions shade_hit evaluated per hit before: pow(roughness, 1.85) * 0.238 (:571) and
// asin(out_n / in_n) of the dielectric TIR test (fresnel.h:34) for both sides of the surface.
__global__ __launch_bounds__(PT_BLOCK) void material_consts_kernel(DevMaterial* mats, int n, float air_n) {
    const int i = blockIdx.x * PT_BLOCK + threadIdx.x;
    if (i >= n) return;
    DevMaterial& m = mats[i];
    m.rough_alpha = pow_pt(m.roughness, 1.85f) * 0.238f;
    m.tir_front = asin_pt(m.refraction_index / air_n);
    m.tir_back = asin_pt(air_n / m.refraction_index);
}

hipError_t launch_material_consts(DevMaterial* mats, int n, float air_n, hipStream_t stream) {
    if (n <= 0 || !mats) return hipSuccess;
    hipLaunchKernelGGL(material_consts_kernel, dim3((n + PT_BLOCK - 1) / PT_BLOCK), dim3(PT_BLOCK), 0, stream, mats, n,
                       air_n);
    return hipGetLastError();
}

// Interactive refit of one mesh (pt_mesh_set_transform; Core/triangle_mesh.cpp:271-328, Bvh/bvh.cpp:
// 332-356): thread i re-transforms mesh-local triangle i into the resident triangle records (edges of
// triangle::intersect as translate_scene computes them, normals into tri_shade) and refits node i's box
// from its initial corners. pt_glm.h keeps glm's operation order, so the result equals the host
// builder's pt_scene_builder_set_transform bit for bit.
__global__ __launch_bounds__(PT_BLOCK) void mesh_refit_kernel(const float4* __restrict__ local, int tri_start,
                                                              int tri_count, const float4* __restrict__ init_nodes,
                                                              int node_first, int node_count, ptglm::M4 T, ptglm::M4 Tn,
                                                              ptglm::M4 C, float4* tri_geom, float4* tri_shade,
                                                              float4* nodes) {
    using namespace ptglm;
    const int i = blockIdx.x * PT_BLOCK + threadIdx.x;
    if (i < tri_count) {
        float v[3][3], n[3][3];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const float4 lv = local[6 * (size_t)i + k], ln = local[6 * (size_t)i + 3 + k];
            const V4 wv = mat_vec(T, V4{lv.x, lv.y, lv.z, 1.0f});
            const V4 wn = mat_vec(Tn, V4{ln.x, ln.y, ln.z, 0.0f});
            v[k][0] = wv.x; v[k][1] = wv.y; v[k][2] = wv.z;
            normalize3(wn.x, wn.y, wn.z, n[k]);
        }
        const size_t t = (size_t)tri_start + i;
        tri_geom[3 * t] = make_float4(v[0][0], v[0][1], v[0][2], 0.0f);
        tri_geom[3 * t + 1] = make_float4(v[1][0] - v[0][0], v[1][1] - v[0][1], v[1][2] - v[0][2], 0.0f);
        tri_geom[3 * t + 2] = make_float4(v[2][0] - v[0][0], v[2][1] - v[0][1], v[2][2] - v[0][2], 0.0f);
        float4 s2 = tri_shade[4 * t + 2];
        tri_shade[4 * t] = make_float4(n[0][0], n[0][1], n[0][2], n[1][0]);
        tri_shade[4 * t + 1] = make_float4(n[1][1], n[1][2], n[2][0], n[2][1]);
        s2.x = n[2][2];
        tri_shade[4 * t + 2] = s2;
    }
    if (i < node_count) {
        const float4 lb = init_nodes[2 * (size_t)i], rt = init_nodes[2 * (size_t)i + 1];
        const V4 a = mat_vec(C, V4{lb.x, lb.y, lb.z, 1.0f});
        const V4 b = mat_vec(C, V4{rt.x, rt.y, rt.z, 1.0f});
        const size_t k = 2 * ((size_t)node_first + i);
        float4 na = nodes[k], nb = nodes[k + 1];
        na.x = a.x; na.y = a.y; na.z = a.z;
        nb.x = b.x; nb.y = b.y; nb.z = b.z;
        nodes[k] = na;
        nodes[k + 1] = nb;
    }
}

hipError_t launch_mesh_refit(const float4* local, int tri_start, int tri_count, const float4* init_nodes, int node_first,
                             int node_count, const ptglm::M4& T, const ptglm::M4& Tn, const ptglm::M4& C,
                             float4* tri_geom, float4* tri_shade, float4* nodes, hipStream_t stream) {
    const int n = tri_count > node_count ? tri_count : node_count;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mesh_refit_kernel, dim3((n + PT_BLOCK - 1) / PT_BLOCK), dim3(PT_BLOCK), 0, stream, local,
                       tri_start, tri_count, init_nodes, node_first, node_count, T, Tn, C, tri_geom, tri_shade, nodes);
    return hipGetLastError();
}

// Diagnostic: the device transcendentals on an array (bitwise check against the oracle's).
__global__ __launch_bounds__(PT_BLOCK) void math_eval_kernel(int which, const float* x, int n, float* o0, float* o1) {
    int i = blockIdx.x * PT_BLOCK + threadIdx.x;
    if (i >= n) return;
    float a = x[i], r0 = 0.0f, r1 = 0.0f;
    switch (which) {
        case 0: sincos_pt(a, &r0, &r1); break;
        case 1: r0 = exp_pt(a); break;
        case 2: r0 = log_pt(a); break;
        case 3: r0 = atan_pt(a); break;
        case 4: r0 = asin_pt(a); break;
        case 5: r0 = acos_pt(a); break;
        case 6: r0 = pow_pt(a, 1.85f); break;
        case 7: r0 = tan_pt(a); break;
        case 8: r0 = sqrtf(a); r1 = 1.0f / a; break;
        case 9: r0 = u8_unit((unsigned int)a); break;  // texel byte -> [0, 1] (texture.h:47-66)
        case 10: r0 = rcp_exact(a); r1 = 1.0f / a; break;
        default: break;
    }
    o0[i] = r0;
    o1[i] = r1;
}

hipError_t launch_math_eval(int which, const float* x, int n, float* o0, float* o1, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(math_eval_kernel, dim3((n + PT_BLOCK - 1) / PT_BLOCK), dim3(PT_BLOCK), 0, stream, which, x, n,
                       o0, o1);
    return hipGetLastError();
}

// ---- thread_shrink (Kernel/parallel_function.cu:42-49): stable remove_if(v < 0) -----------
// Three passes over 256-element tiles: per-tile survivor counts (wave ballots), an exclusive
// scan of the tile counts in one workgroup, then a stable scatter into a scratch array.
__global__ __launch_bounds__(256) void shrink_count_kernel(const int* in, int n, int* tile_counts) {
    __shared__ int wave_cnt[4];
    int i = blockIdx.x * 256 + threadIdx.x;
    bool keep = i < n && in[i] >= 0;
    unsigned long long m = __ballot(keep);
    if ((threadIdx.x & 63) == 0) wave_cnt[threadIdx.x >> 6] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) tile_counts[blockIdx.x] = wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
}

__global__ __launch_bounds__(1024) void shrink_scan_kernel(int* tile_counts, int tiles, int* total) {
    __shared__ int part[1024];
    // each thread scans a contiguous chunk, then the chunk sums are scanned in LDS
    int per = (tiles + 1023) / 1024;
    int begin = threadIdx.x * per;
    int end = min(begin + per, tiles);
    int s = 0;
    for (int i = begin; i < end; i++) s += tile_counts[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        int v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int run = part[threadIdx.x] - s;  // exclusive prefix of this chunk
    for (int i = begin; i < end; i++) {
        int c = tile_counts[i];
        tile_counts[i] = run;
        run += c;
    }
    if (threadIdx.x == 1023) *total = part[1023];
}

__global__ __launch_bounds__(256) void shrink_scatter_kernel(const int* in, int n, const int* tile_offsets, int* out) {
    __shared__ int wave_cnt[4];
    int i = blockIdx.x * 256 + threadIdx.x;
    int v = i < n ? in[i] : -1;
    bool keep = i < n && v >= 0;
    unsigned long long m = __ballot(keep);
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) wave_cnt[w] = __popcll(m);
    __syncthreads();
    int base = tile_offsets[blockIdx.x];
    for (int k = 0; k < w; k++) base += wave_cnt[k];
    unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    if (keep) out[base + __popcll(m & lt)] = v;
}

// ---- host-side launchers ------------------------------------------------------------------
int env_int(const char* name, int dflt, int lo, int hi) {
    const char* e = getenv(name);
    int v = e ? atoi(e) : dflt;
    return v < lo ? lo : (v > hi ? hi : v);
}

using PassFn = void (*)(const LaunchParams*, int, int, int, int);

// QN (quantised nodes) only for leaf size 1 and the uninstrumented kernel: the instrumented kernel
// walks the exact nodes so its visit counts are the reference's.
static PassFn pass_fn(bool leaf1, bool stats, int minw, bool qn) {
    if (leaf1 && !stats) {
        if (qn) {
            if (minw == 6) return pass_kernel<true, false, 6, true>;
            if (minw == 7) return pass_kernel<true, false, 7, true>;
            if (minw == 8) return pass_kernel<true, false, 8, true>;
            return pass_kernel<true, false, 5, true>;
        }
        if (minw == 4) return pass_kernel<true, false, 4, false>;
        if (minw == 6) return pass_kernel<true, false, 6, false>;
        if (minw == 7) return pass_kernel<true, false, 7, false>;
        if (minw == 8) return pass_kernel<true, false, 8, false>;
        return pass_kernel<true, false, 5, false>;
    }
    if (leaf1 && stats) return pass_kernel<true, true, 5, false>;
    if (!stats) return pass_kernel<false, false, 5, false>;
    return pass_kernel<false, true, 5, false>;
}

// PT_MIN_WAVES overrides the occupancy target: 8 waves/SIMD for pass_kernel (64 VGPRs); for pass_kernel_u
// 7 when the scene reaches no participating medium (72 VGPRs: no spills without textures, +3.5 % over 6 on
// the bench frame; one cold spill with textures, +6.7 % on C5) and 6 otherwise (80 VGPRs; at 72 the medium
// step spills: C4 5049 vs 5378 Mrays/s, profiles/r02/workloads).
int pass_min_waves(bool unified, int feat) {
    static int w = [] {
        const char* e = getenv("PT_MIN_WAVES");
        int v = e ? atoi(e) : 0;
        return (v >= 4 && v <= 8) ? v : 0;
    }();
    if (w) return w;
    if (!unified) return 8;
    return (feat & PT_FEAT_MEDIUM) ? 6 : 7;
}

// PT_UNIFIED=0 selects pass_kernel for the default configuration (leaf size 1, uninstrumented, exact
// nodes); otherwise pass_kernel_u runs it. PT_SHADE_MIN / PT_WALK_STEPS tune pass_kernel_u.
bool unified_enabled() {
    static const int on = env_int("PT_UNIFIED", 1, 0, 1);
    return on != 0;
}

using PassFnU = void (*)(const LaunchParams*, int, int, int, int, int, int, int, int, int);

// The product configuration specialised on the scene's features (pt_path.h PT_FEAT_*): feat is what the
// scene can reach; PT_FEAT_SPECIALISE=0 keeps the all-features kernel.
static PassFnU pass_fn_feat(int minw, int feat, int pool) {
    static const int spec = env_int("PT_FEAT_SPECIALISE", 1, 0, 1);
    if (!spec) feat = PT_FEAT_ALL;
    // tail pool: the bench scene's instance, else the all-features one
    if (pool && minw == 7 && feat == 0) return pass_kernel_u<7, false, false, 2, true, false, 0, true>;
    if (pool) return pass_kernel_u<6, false, false, 2, true, false, PT_FEAT_ALL, true>;
    switch (minw * 4 + feat) {
        case 5 * 4 + 0: return pass_kernel_u<5, false, false, 2, true, false, 0>;
        case 5 * 4 + 1: return pass_kernel_u<5, false, false, 2, true, false, 1>;
        case 5 * 4 + 2: return pass_kernel_u<5, false, false, 2, true, false, 2>;
        case 6 * 4 + 0: return pass_kernel_u<6, false, false, 2, true, false, 0>;
        case 6 * 4 + 1: return pass_kernel_u<6, false, false, 2, true, false, 1>;
        case 6 * 4 + 2: return pass_kernel_u<6, false, false, 2, true, false, 2>;
        case 7 * 4 + 0: return pass_kernel_u<7, false, false, 2, true, false, 0>;
        case 7 * 4 + 1: return pass_kernel_u<7, false, false, 2, true, false, 1>;
        case 7 * 4 + 2: return pass_kernel_u<7, false, false, 2, true, false, 2>;
        case 8 * 4 + 0: return pass_kernel_u<8, false, false, 2, true, false, 0>;
        case 8 * 4 + 1: return pass_kernel_u<8, false, false, 2, true, false, 1>;
        default: break;
    }
    return nullptr;
}

// PT_WALK_CHAIN: records per binary walk step (walk_box_chain); 1 = walk_box. wide: the scene has wide
// records and PT_WIDE (default 0) allows their walk (walk_wide). feat: the scene's reachable features.
static PassFnU pass_fn_u(int minw, bool qn, bool wide, int feat, int pool) {
    static const int prof = env_int("PT_UPROF", 0, 0, 1);
    static const int chain = env_int("PT_WALK_CHAIN", 2, 1, 3);
    static const int pf = env_int("PT_TRI_PREFETCH", 1, 0, 1);
    if (prof && pool && !qn && !wide)
        return pass_kernel_u<6, true, false, 2, true, false, PT_FEAT_ALL, true>;
    if (prof) return qn ? pass_kernel_u<6, true, true, 1, false, false>
                        : (wide ? pass_kernel_u<6, true, false, 2, true, true> : pass_kernel_u<6, true, false, 2, true, false>);
    if (qn) return minw == 6 ? pass_kernel_u<6, false, true, 1, false, false> : pass_kernel_u<5, false, true, 1, false, false>;
    if (wide) return minw == 5 ? pass_kernel_u<5, false, false, 2, true, true> : pass_kernel_u<6, false, false, 2, true, true>;
    if (chain == 1) return minw == 6 ? pass_kernel_u<6, false, false, 1, false, false> : pass_kernel_u<5, false, false, 1, false, false>;
    if (chain == 3) return minw == 6 ? pass_kernel_u<6, false, false, 3, false, false> : pass_kernel_u<5, false, false, 3, false, false>;
    if (pf) {  // specialised on the scene's features, or with the tail pool (nullptr: neither applies)
        PassFnU f = pass_fn_feat(minw, feat, pool);
        if (f) return f;
    }
    if (pf) return minw == 7 ? pass_kernel_u<7, false, false, 2, true, false>
                             : (minw == 6 ? pass_kernel_u<6, false, false, 2, true, false> : pass_kernel_u<5, false, false, 2, true, false>);
    return minw == 6 ? pass_kernel_u<6, false, false, 2, false, false> : pass_kernel_u<5, false, false, 2, false, false>;
}

// pass_kernel_u keeps every material and sphere in LDS: scenes whose tables exceed PT_LDS_TABLES bytes
// (about 256 materials and 256 spheres) run pass_kernel.
#define PT_LDS_TABLES (32 * 1024)
static bool use_unified(bool leaf1, bool stats, bool qn, int lds_bytes) {
    (void)qn;
    return leaf1 && !stats && unified_enabled() && lds_bytes <= PT_LDS_TABLES;
}

static bool regroup_applies(bool leaf1, bool stats, bool qn, bool wide, int lds_bytes) {
    return use_unified(leaf1, stats, qn, lds_bytes) && !qn && !wide;
}

// pass_kernel_r's wave split: PT_RG_WAVES = 10 * walkers + shaders (52: five walker waves and two
// shader waves per workgroup of 448 lanes). MINW as pass_kernel_u: 7 without textures and media, else 6.
struct RgKernel {
    PassFnU fn;
    int threads;
};
static RgKernel pass_fn_r(int feat) {
    static const int split = env_int("PT_RG_WAVES", 52, 11, 99);
    static const int prof = env_int("PT_UPROF", 0, 0, 1);
    const bool plain = feat == 0;
    if (prof) return {pass_kernel_r<7, 5, 2, true, 0>, 7 * 64};
    switch (split) {
        case 31: return {plain ? pass_kernel_r<7, 3, 1, false, 0> : pass_kernel_r<6, 3, 1, false, PT_FEAT_ALL>, 4 * 64};
        case 61: return {plain ? pass_kernel_r<7, 6, 1, false, 0> : pass_kernel_r<6, 6, 1, false, PT_FEAT_ALL>, 7 * 64};
        case 43: return {plain ? pass_kernel_r<7, 4, 3, false, 0> : pass_kernel_r<6, 4, 3, false, PT_FEAT_ALL>, 7 * 64};
        case 21: return {plain ? pass_kernel_r<7, 2, 1, false, 0> : pass_kernel_r<6, 2, 1, false, PT_FEAT_ALL>, 3 * 64};
        default: return {plain ? pass_kernel_r<7, 5, 2, false, 0> : pass_kernel_r<6, 5, 2, false, PT_FEAT_ALL>, 7 * 64};
    }
}

hipError_t launch_pass(const LaunchParams* params_dev, const PassChoice& pc, int first_pass, int batch_log2,
                       int write_u8, int grid, int lds_bytes, hipStream_t stream) {
    const bool leaf1 = pc.leaf1, qn = pc.qn, wide = pc.wide, stats = pc.stats;
    const int feat = pc.feat;
    if (pc.regroup && regroup_applies(leaf1, stats, qn, wide, lds_bytes)) {
        // PT_RG_HANDOFF / PT_RG_WALK_MIN: a walker wave hands its ready paths over once this many are
        // ready or at most this many lanes still walk; PT_RG_BATCH / PT_RG_SPIN: a shader wave shades
        // once this many paths wait, or after this many idle rounds with fewer
        static const int chunk = env_int("PT_CHUNK_MEGA", 64, 0, 4096);
        static const int handoff = env_int("PT_RG_HANDOFF", 16, 1, 64);
        static const int walk_steps = env_int("PT_WALK_STEPS", 8, 1, 64);
        static const int tri_min = env_int("PT_TRI_MIN", 6, 1, 64);
        static const int walk_min = env_int("PT_RG_WALK_MIN", 40, 0, 64);
        static const int batch = env_int("PT_RG_BATCH", 48, 1, 64);
        static const int spin = env_int("PT_RG_SPIN", 8, 0, 0xffff);
        const RgKernel k = pass_fn_r(feat);
        const LaunchParams* a0 = params_dev;
        int a1 = first_pass, a2 = write_u8, a3 = chunk, a4 = batch_log2, a5 = handoff, a6 = walk_steps, a7 = tri_min,
            a8 = walk_min, a9 = spin | (batch << 16);
        void* args[] = {&a0, &a1, &a2, &a3, &a4, &a5, &a6, &a7, &a8, &a9};
        hipError_t e = hipLaunchKernel((const void*)k.fn, dim3(grid), dim3(k.threads), args, (size_t)lds_bytes, stream);
        if (e != hipSuccess) return e;
        return hipGetLastError();
    }
    if (use_unified(leaf1, stats, qn, lds_bytes)) {
        // 64-unit chunks and a 28-lane shading batch: measured best with frames in flight
        static const int chunk = env_int("PT_CHUNK_MEGA", 64, 0, 4096);
        static const int shade_min = env_int("PT_SHADE_MIN", 28, 1, 64);
        static const int walk_steps = env_int("PT_WALK_STEPS", 8, 1, 64);
        const LaunchParams* a0 = params_dev;
        // measured best with frames in flight; lanes with a deferred leaf walk on, so their batches wait longer
        static const int tri_min = env_int("PT_TRI_MIN", PT_DEFER ? 16 : 6, 1, 64);
        static const int walk_min = env_int("PT_WALK_MIN", 8, 0, 64);
        // PT_TAIL_SHADE_MIN / PT_TAIL_WALK_MIN: the shading thresholds of a wave once the work is drained
        static const int tail_shade = env_int("PT_TAIL_SHADE_MIN", shade_min, 1, 64);
        static const int tail_walk = env_int("PT_TAIL_WALK_MIN", walk_min, 0, 64);
        const int tail_pool = pc.tail_pool < 0 ? 0 : (pc.tail_pool > 64 ? 64 : pc.tail_pool);
        int a1 = first_pass, a2 = write_u8, a3 = chunk, a4 = batch_log2, a5 = shade_min, a6 = walk_steps, a7 = tri_min,
            a8 = walk_min, a9 = tail_shade | (tail_walk << 8) | (tail_pool << 16);
        void* args[] = {&a0, &a1, &a2, &a3, &a4, &a5, &a6, &a7, &a8, &a9};
        hipError_t e = hipLaunchKernel((const void*)pass_fn_u(pass_min_waves(true, feat), qn, wide && !qn, feat, tail_pool),
                                       dim3(grid), dim3(PT_UBLOCK), args,
                                       (size_t)lds_bytes, stream);
        if (e != hipSuccess) return e;
        return hipGetLastError();
    }
    PassFn fn = pass_fn(leaf1, stats, pass_min_waves(false, feat), qn);
    const LaunchParams* a0 = params_dev;
    static const int chunk = env_int("PT_CHUNK_MEGA", 32, 0, 4096);
    int a1 = first_pass, a2 = write_u8, a3 = chunk, a4 = batch_log2;
    void* args[] = {&a0, &a1, &a2, &a3, &a4};
    hipError_t e = hipLaunchKernel((const void*)fn, dim3(grid), dim3(PT_BLOCK), args, 0, stream);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t launch_accumulate(const LaunchParams* params_dev, int units, int first_pass, int batch_log2, int write_u8,
                             hipStream_t stream) {
    if (units <= 0) return hipSuccess;
    hipLaunchKernelGGL(accumulate_kernel, dim3((units + PT_BLOCK - 1) / PT_BLOCK), dim3(PT_BLOCK), 0, stream,
                       params_dev, first_pass, batch_log2, write_u8);
    return hipGetLastError();
}

hipError_t launch_u8(const DevConfig& cfg, const float* image, uint8_t* image256, int pixel_count, int pass,
                     hipStream_t stream) {
    if (pixel_count <= 0) return hipSuccess;
    int grid = (pixel_count + PT_BLOCK - 1) / PT_BLOCK;
    hipLaunchKernelGGL(u8_kernel, dim3(grid), dim3(PT_BLOCK), 0, stream, cfg, image, image256, pixel_count, pass);
    return hipGetLastError();
}

// The pass kernel launch_pass picks for these arguments, as text (bench.py's roofline.kernel).
std::string pass_kernel_desc(const PassChoice& pc, int lds_bytes) {
    const bool leaf1 = pc.leaf1, qn = pc.qn, wide = pc.wide, stats = pc.stats;
    const int feat = pc.feat;
    char buf[160];
    if (pc.regroup && regroup_applies(leaf1, stats, qn, wide, lds_bytes)) {
        static const int split = env_int("PT_RG_WAVES", 52, 11, 99);
        const int s = (split == 31 || split == 61 || split == 43 || split == 21) ? split : 52;
        std::snprintf(buf, sizeof(buf), "pass_kernel_r<MINW=%d,NWALK=%d,NSHADE=%d,FEAT=%d>", feat == 0 ? 7 : 6, s / 10,
                      s % 10, feat == 0 ? 0 : PT_FEAT_ALL);
    } else if (use_unified(leaf1, stats, qn, lds_bytes)) {
        static const int spec = env_int("PT_FEAT_SPECIALISE", 1, 0, 1);
        static const int chain = env_int("PT_WALK_CHAIN", 2, 1, 3);
        static const int pf = env_int("PT_TRI_PREFETCH", 1, 0, 1);
        const int pool = pc.tail_pool;
        int minw = pass_min_waves(true, feat);
        // the instance pass_fn_u picks for this wave target (not every variant has every target)
        if (qn || (chain != 2 && !wide) || (!pf && !wide)) minw = minw == 6 ? 6 : 5;
        else if (wide) minw = minw == 5 ? 5 : 6;
        int f = spec && !qn && !wide && pf && chain == 2 ? feat : PT_FEAT_ALL;
        const bool tp = pool > 0 && !qn && !wide && pf && chain == 2;
        if (tp && !(minw == 7 && f == 0)) { minw = 6; f = PT_FEAT_ALL; }  // pass_fn_feat's tail-pool instances
        std::snprintf(buf, sizeof(buf), "pass_kernel_u<MINW=%d,QN=%d,CHAIN=%d,PF=%d,WIDE=%d,FEAT=%d%s>", minw,
                      qn ? 1 : 0, qn ? 1 : chain, qn ? 0 : pf, wide && !qn ? 1 : 0, f, tp ? ",TAILPOOL" : "");
    } else {
        std::snprintf(buf, sizeof(buf), "pass_kernel<LEAF1=%d,STATS=%d,MINW=%d,QN=%d>", leaf1 ? 1 : 0, stats ? 1 : 0,
                      pass_min_waves(false, feat), qn ? 1 : 0);
    }
    return buf;
}

int pass_grid_size(const PassChoice& pc, int lds_bytes) {
    const bool leaf1 = pc.leaf1, qn = pc.qn, wide = pc.wide, stats = pc.stats, regroup = pc.regroup;
    const int feat = pc.feat;
    int dev = 0, cus = 0, blocks = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    if (regroup && regroup_applies(leaf1, stats, qn, wide, lds_bytes)) {
        const RgKernel k = pass_fn_r(feat);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, (const void*)k.fn, k.threads, (size_t)lds_bytes) !=
                hipSuccess || blocks <= 0)
            blocks = 1;
        return cus * blocks;
    }
    const bool u = use_unified(leaf1, stats, qn, lds_bytes);
    const void* fn = u ? (const void*)pass_fn_u(pass_min_waves(true, feat), qn, wide && !qn, feat, pc.tail_pool)
                       : (const void*)pass_fn(leaf1, stats, pass_min_waves(false, feat), qn);
    const size_t lds = u ? (size_t)lds_bytes : 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, u ? PT_UBLOCK : PT_BLOCK, lds) != hipSuccess || blocks <= 0) blocks = u ? 4 * PT_BLOCK / PT_UBLOCK : 4;
    if (cus <= 0) cus = 256;
    return cus * blocks;
}

hipError_t shrink(int* data, int n, int* scratch, int* tile_counts, int* total_dev, int* total_host, hipStream_t stream) {
    if (n <= 0) { *total_host = 0; return hipSuccess; }
    int tiles = (n + 255) / 256;
    hipLaunchKernelGGL(shrink_count_kernel, dim3(tiles), dim3(256), 0, stream, data, n, tile_counts);
    hipLaunchKernelGGL(shrink_scan_kernel, dim3(1), dim3(1024), 0, stream, tile_counts, tiles, total_dev);
    hipLaunchKernelGGL(shrink_scatter_kernel, dim3(tiles), dim3(256), 0, stream, data, n, tile_counts, scratch);
    hipError_t e = hipMemcpyAsync(total_host, total_dev, sizeof(int), hipMemcpyDeviceToHost, stream);
    if (e != hipSuccess) return e;
    e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return e;
    if (*total_host > 0) {
        e = hipMemcpyAsync(data, scratch, (size_t)*total_host * sizeof(int), hipMemcpyDeviceToDevice, stream);
        if (e != hipSuccess) return e;
        e = hipStreamSynchronize(stream);
    }
    return e;
}

}  // namespace pt
