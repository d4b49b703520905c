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

// One path per feature: the measured alternatives of rounds 4-5 (refill-time path generation, struct copies of the
// launch parameters, threadIdx-held lane indices) and the diagnostic phase duplicates (tools/build_dup.sh) live as
// patches under profiles/ (profiles/r06/pruned/), not as preprocessor arms here.

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

// pass_kernel_u reads its configuration, tiling and output fields where it uses them (const_ref) instead of copying
// the three structs at the top of every round. At 8 waves per SIMD a wave has about 80 SGPRs, so the copies did not
// fit: every round reloaded ~30 dwords and spilled them into VGPR lanes again (29 v_writelane and eight scalar-load
// waits per round, 4.8 M rounds per launch), and every use read them back (v_readlane). Read at their uses they live
// for a few instructions: v_readlane 284 -> 59, v_writelane 74 -> 46 in the bench kernel; metric 15411-15433 vs
// 15028-15144 Mrays/s (profiles/r05/lazy/ab.txt).
// A reference to *p whose loads go through the constant address space wherever they are used (the generic
// pointer is an address-space cast of a constant one, which the compiler's address-space inference sees
// through once everything is inlined): the fields are read at their uses, not copied at one point.
template <class T>
__device__ __forceinline__ const T& const_ref(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(4))) const T ConstT;
    return *(const T*)(const ConstT*)(unsigned long long)p;
#else
    return *p;
#endif
}

// pass_kernel_u recomputes its lane index where it uses it (two v_mbcnt in a volatile asm, which the compiler neither
// merges nor hoists) and keeps its wave index in an SGPR, instead of holding threadIdx-derived values in VGPRs across
// the loop: at 64 VGPRs they were spilled to scratch and reloaded, with a wait on memory, in the refill and at every
// path's end. No instance spills to scratch now (the bench kernel had 16 B, C5's 12 B); metric 15628-15659 vs
// 15222-15411 Mrays/s (profiles/r05/lane/ab.txt).
__device__ __forceinline__ int lane_now() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
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
template <bool LEAF1, bool STATS, int MINW>
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
                alive = trace_step<LEAF1, STATS>(sc, cfg, depth, pseed, &ps, &ctr);
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
                if (batch_log2 == 0 && !out.via_rad) {
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
// (+2.5 % over starting survivors inside the shading batch, profiles/r02/onesite.txt). Every lane
// still computes exactly the reference sequence for its path (same node order, same tests, same draws
// keyed by (pass, pixel, depth)); only the interleaving between lanes changes.
enum : int { LANE_WANT = 0, LANE_WALK = 1, LANE_READY = 2, LANE_DONE = 3, LANE_TRI = 4, LANE_NEW = 5 };

// Starts the walk of the first mesh at or after `mesh` with a non-empty node range. The ranges of the
// first PT_LDS_MESHES meshes come from the workgroup's LDS copy (lds_mesh, filled at kernel start), the
// rest from global memory (scenes of more than PT_LDS_MESHES meshes).
#define PT_LDS_MESHES 64
typedef int i32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bool start_mesh(const DevScene& sc, const int2* lds_mesh, int& mesh, int2& range) {
    while (mesh < sc.mesh_num) {
        int2 r;
        if (mesh < PT_LDS_MESHES) {
            r = lds_mesh[mesh];
        } else {  // a buffer load (not a pointer select that would turn both into flat loads)
            const i32x2 v = __builtin_bit_cast(i32x2, __builtin_amdgcn_raw_buffer_load_b64(
                make_rsrc(sc.mesh_range, sc.mesh_num * 8), mesh * 8, 0, 0));
            r.x = v.x; r.y = v.y;
        }
        if (r.x != r.y) {
            range = r;
            return true;
        }
        mesh++;
    }
    return false;
}

// start_mesh for scenes of at most PT_LDS_MESHES meshes: lds_next[m] holds the range and index of the
// first non-empty mesh at or after m (index mesh_num and an empty range: none left), built at kernel
// start. One LDS read and no loop: a mesh change in a walk step then waits only on LDS, not on the wave's
// outstanding vector loads (the looping version's mixed LDS / buffer-load path made it wait for every
// one, parked lanes' triangle prefetches included).
__device__ __forceinline__ bool start_mesh_next(const int4* lds_next, int& mesh, int2& range) {
    const int4 e = lds_next[mesh];
    mesh = e.z;
    range = make_int2(e.x, e.y);
    return e.x != e.y;
}

// A mesh walk's start state over node range r (the walk's local min_t starts at infinity; at the segment's
// medium bound in the medium-bounded mode, pt_path.h medium_bound).
__device__ __forceinline__ void walk_start(MeshWalk& w, int2 r, float t0 = __builtin_inff()) {
    w.pos = r.x; w.end = r.y;
    w.t = t0; w.t1 = 0.0f; w.t2 = 0.0f; w.tri = -1;
}

// ---- root boxes at segment start (at most PT_ROOT_MESHES meshes) ----------------------------------
// Each mesh's walk starts at its root with a local min_t of infinity (intersect_triangle_mesh_bvh,
// :113-150), so a ray whose slab test fails on a mesh's root box gets nothing from that mesh. The roots of
// the first PT_ROOT_MESHES meshes are kept in LDS; a segment tests them all at its start and walks only the
// meshes whose root passes, starting below a passing internal root (the test there would repeat the same
// test with the same infinite min_t). `mesh` then holds the mesh being walked in bits 0-7 and the meshes
// still to walk as a bit mask from bit 8 on (bit 8 + i: mesh i), so the skip costs no register.
#define PT_ROOT_MESHES 24
__device__ __forceinline__ int2 root_walk_range(const int2* lds_mesh, const float4* lds_root, int m) {
    const int2 r = lds_mesh[m];
    return make_int2(f2i(lds_root[2 * m + 1].w) < 0 ? r.x + 1 : r.x, r.y);  // below an internal root, at a leaf root
}

// Start of one trace_ray_kernel invocation (path_tracer_kernel.cu:418-454): brute-force spheres into
// the closest hit, then the walk of the first mesh (roots, wave-uniform: of the first mesh whose root box
// the ray hits, from the LDS root table). Both ways produce only the first mesh and its node range, and
// the walk state is set once from them, so the compiler merges no walk fields between the two.
__device__ __forceinline__ int begin_segment(const DevScene& sc, bool roots, const int2* lds_mesh,
                                             const float4* lds_root, const PathState& ps, v3& inv, Hit& h,
                                             MeshWalk& w, int& mesh, float t0 = __builtin_inff()) {
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
    int first = sc.first_mesh;
    int2 range = sc.first_range;
    bool any = true;
    if (roots) {
        unsigned int todo = 0;
        for (int i = sc.first_mesh; i < sc.mesh_num; i++) {  // wave-uniform loop, broadcast LDS reads
            const int2 r = lds_mesh[i];
            if (r.x == r.y) continue;
            float entry;
            if (box_hit(lds_root[2 * i], lds_root[2 * i + 1], ps.o, inv, &entry) && entry <= t0)
                todo |= 1u << i;
        }
        any = todo != 0u;
        const int m = any ? __builtin_ctz(todo) : 0;
        first = m | (int)((todo & (todo - 1u)) << 8);
        range = root_walk_range(lds_mesh, lds_root, m);
    }
    mesh = first;
    walk_start(w, range, t0);
    return any ? LANE_WALK : LANE_READY;
}
// The next mesh of a root-masked segment (mesh_done) and its walk range: false when none is left.
__device__ __forceinline__ bool next_root_mesh(const int2* lds_mesh, const float4* lds_root, int& mesh, int2& range) {
    const unsigned int rest = (unsigned int)mesh >> 8;
    const int m = rest ? __builtin_ctz(rest) : 0;
    range = root_walk_range(lds_mesh, lds_root, m);
    mesh = m | (int)((rest & (rest - 1u)) << 8);
    return rest != 0u;
}

// pixel_256_transform_gamma_corrected_kernel (:644-680) for one finished (pixel, pass) unit
// depth: the path's ray segments, counted into its band when the context measures band costs.
__device__ __forceinline__ unsigned int frame_local(unsigned int u, unsigned int frame_units) {
    while (u >= frame_units) u -= frame_units;
    return u;
}

// unit: the launch's unit (pass_rad index). frame_units: the units of one frame copy of a pt_render_frames launch
// (0 for a launch of one frame); the unit within its frame copy is derived only where it is used (band costs, the
// direct image path): the MULTI launches write pass_rad by the launch's unit, and the subtraction loop over the
// frame copies, run for every finished path, cost up to G iterations per shading batch (round 5)
__device__ __forceinline__ void finish_unit(const DevTiling& til, const DevConfig& cfg, const DevOutput& out,
                                            const PathState& ps, unsigned int unit, unsigned int frame_units,
                                            int first_pass, int write_u8, int batch_log2, float clamp_hi, int depth) {
    if (til.band_cost) {
        const unsigned int lu = frame_units ? frame_local(unit, frame_units) : unit;
        atomicAdd(&til.band_cost[pixel_band(til, unit_to_pixel(til, lu >> batch_log2))], (unsigned int)depth);
    }
    const v3 c = clamp3(ps.rad, 0.0f, clamp_hi);
    if (batch_log2 == 0 && !out.via_rad) {  // (never for several frame copies: they go through pass_rad)
        const int pixel = unit_to_pixel(til, unit);  // one frame copy here: the unit is its own frame's
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

// ---- the generation ring --------------------------------------------------------------------------------------
// generate_ray_kernel (:299-379) runs once per new path. Generated where a refill hands out units, it executes
// with only the refilled lanes active: 9.2 of 64 on the metric frame, 7 % of the kernel's VALU (round 4's phase
// split, tools/build_dup.sh). Here a wave that runs out of generated paths fetches its next chunk of units (one returning atomic, as
// before) and ALL its lanes generate the chunk's camera paths at once, lane i unit i, into the wave's 64-entry
// ring in LDS; refills then pop entries in lane order. An entry is 32 B: {origin, path seed} {direction, unit}.
// The other per-path fields are constants at generation (throughput 1, radiance 0, air, depth 0). Every path is
// still the generate_path of its (pass, pixel): only which instruction serves it changes.
#define PT_RING 64
__device__ __forceinline__ void gen_ring_put(float4* ring, int e, const PathState& ps, int32_t pseed, unsigned int unit) {
    ring[2 * e] = make_float4(ps.o.x, ps.o.y, ps.o.z, __int_as_float(pseed));
    ring[2 * e + 1] = make_float4(ps.d.x, ps.d.y, ps.d.z, __uint_as_float(unit));
}
__device__ __forceinline__ void gen_ring_get(const float4* ring, int e, PathState& ps, int32_t& pseed, unsigned int& unit) {
    const float4 a = ring[2 * e], b = ring[2 * e + 1];
    ps.o = mk3(a.x, a.y, a.z);
    ps.d = mk3(b.x, b.y, b.z);
    ps.thr = mk3(1.0f, 1.0f, 1.0f);
    ps.rad = mk3(0.0f, 0.0f, 0.0f);
    ps.medium = -1;
    pseed = __float_as_int(a.w);
    unit = __float_as_uint(b.w);
}

// PROF: wave-level occupancy counters of the state machine into stats[16..31] (tools/uprof.py):
// rounds, walk steps, walking lanes summed over steps, shading batches, lanes shaded, triangle
// batches, lanes in triangle batches, lanes refilled, then cycles and the drained/ready/idle counts,
// and the launch timeline in stats[32..41].
// FEAT: the scene features shade_hit can reach (pt_path.h PT_FEAT_*).
// MULTI: the pt_render_frames instance (several frames per launch: a ring fill that spans frames generates them one
// frame at a time); the single-frame instances go without that loop
template <int MINW, bool PROF, int FEAT, bool MULTI = false>
__global__ __launch_bounds__(PT_UBLOCK, MINW) void pass_kernel_u(const LaunchParams* __restrict__ params, int first_pass,
                                                                int write_u8, int chunk, int batch_log2, int shade_min,
                                                                int walk_steps, int tri_min, int walk_min) {
    // the wave's index in the workgroup, wave-uniform (an SGPR); the lane index is recomputed at each use
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#define PT_LANE lane_now()
#define PT_TID (wave * 64 + lane_now())
    const LaunchParams* P0 = params;
    // workgroup copies in LDS: the first mesh ranges, every material and every sphere (the launch
    // reserves their bytes of dynamic LDS; pass_kernel_u runs only when that fits, PT_LDS_TABLES)
    __shared__ int2 lds_mesh[PT_LDS_MESHES];
    __shared__ int4 lds_next[PT_LDS_MESHES + 1];
    __shared__ float4 lds_root[2 * PT_ROOT_MESHES];
    __shared__ float4 lds_ring[PT_UBLOCK / 64][2 * PT_RING];  // one generation ring per wave
    float4* ring = lds_ring[wave];
    int ring_head = 0, ring_end = 0;  // wave-uniform: entries [ring_head, ring_end) are generated, not yet taken
    // the lane's (pixel, pass) unit lives in LDS: it is read once, at the path's end (finish_unit), and held in a
    // VGPR it was spilled to scratch around the ring fill (written back after every shading batch: 0.6 GB of
    // scratch writes per launch)
    __shared__ unsigned int lds_unit[PT_UBLOCK];
    extern __shared__ float4 lds_dyn[];
    DevMaterial* lds_mats = reinterpret_cast<DevMaterial*>(lds_dyn);
    {
        const int2* mr = uniform_ptr(P0->sc.mesh_range);
        const int n = min(uniform_int(P0->sc.mesh_num), PT_LDS_MESHES);
        for (int i = threadIdx.x; i < n; i += PT_UBLOCK) lds_mesh[i] = mr[i];
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
            if (n <= PT_ROOT_MESHES) {  // lds_root (begin_segment with roots)
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
    int32_t pseed = 0;
    int depth = 0;
    int mode = LANE_WANT;
    float wbound = __builtin_inff();  // every mesh walk's starting min_t (PT_FEAT_MBOUND instances only)
    unsigned long long segments = 0;  // wave-uniform: lanes shaded (ray segments traced)
    Counters none = {0u, 0u, 0u, 0u, 0u, 0u};
    // the units of one frame copy; a pt_render_frames launch has `frames` copies one after another
    const unsigned int frame_units = (unsigned int)P0->til.unit_count << batch_log2;
    const unsigned int units = MULTI ? frame_units * (unsigned int)max(1, P0->out.frames) : frame_units;
    const EvenRegions regions{units, (units + PT_SHARDS - 1) / PT_SHARDS};
    WorkCursor cursor = work_begin();
    bool drained = false;
    unsigned long long prof[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tc = 0, tc2 = 0;
    // PROF timeline (stats[32..41]): this wave's start, the refill that first found the work drained,
    // its end (real-time clock), and the paths it shaded after the drain
    unsigned long long t_start = 0, t_drain = 0, tail_segments = 0;
    // PROF: refill rounds that started at least one camera path (the path-generation phase's batches), and
    // wave rounds summed with the lanes holding a path at their start (the control phase's occupancy)
    unsigned long long gen_batches = 0, live_lane_rounds = 0;
    if (PROF) t_start = __builtin_amdgcn_s_memrealtime();
    while (true) {
        const LaunchParams* P = params;
        asm volatile("" : "+s"(P));  // the parameter block's address reloaded each round, not held across it
        P = uniform_ptr(P);
        DevScene sc = load_const(&P->sc);
        sc.materials = lds_mats;
        sc.spheres = lds_spheres;
        const DevConfig& cfg = const_ref(&P->cfg);
        const DevTiling& til = const_ref(&P->til);
        const DevOutput& out = const_ref(&P->out);
        const bool roots = sc.mesh_num <= PT_ROOT_MESHES;  // wave-uniform
        if (PROF) {
            prof[0]++;
            tc = __builtin_readcyclecounter();
            live_lane_rounds += (unsigned long long)__popcll(__ballot(mode != LANE_WANT && mode != LANE_DONE));
        }

        // lanes without a path take the next (pixel, pass) units, one atomic per wave (pt_work.h)
        const bool want = mode == LANE_WANT;
        const unsigned long long need_mask = __ballot(want);
        if (need_mask) {
            // lanes take generated paths from the ring in lane order; when it runs dry the wave fetches the next
            // chunk and generates all of it (gen_ring_fill below), then the remaining lanes take from the new ring
            const int taken = __popcll(need_mask);
            const int rank = count_below(need_mask);
            const int avail = ring_end - ring_head;
            bool got = false;
            unsigned int u = ~0u;
            if (want && rank < avail) {
                gen_ring_get(ring, ring_head + rank, ps, pseed, u);
                got = true;
            }
            if (taken <= avail) {
                ring_head += taken;
            } else if (!drained && work_fetch(out.fetch, regions.stride, regions, (unsigned int)min(chunk, PT_RING),
                                              cursor)) {
                const int n = (int)(cursor.end - cursor.cur);  // <= min(chunk, PT_RING): the ring's bound, on the device
                if (PROF) { prof[7] += (unsigned long long)n; gen_batches++; }
                // gen_ring_fill: lane i generates unit cursor.cur + i. The camera is read through the scalar cache,
                // so a chunk that spans frames (MULTI) is generated one frame at a time
                if (PT_LANE < n) {
                    const unsigned int gu = cursor.cur + (unsigned int)PT_LANE;
                    // the chunk's frames f_lo..f_hi are wave-uniform (scalar arithmetic on the chunk's bounds): one
                    // pass per frame, each lane generating in its own frame's pass (one pass unless the chunk spans
                    // frames)
                    const unsigned int c0 = (unsigned int)__builtin_amdgcn_readfirstlane((int)cursor.cur);
                    const unsigned int f_lo = MULTI ? c0 / frame_units : 0u;
                    const unsigned int f_hi = MULTI ? (c0 + (unsigned int)n - 1u) / frame_units : 0u;
                    for (unsigned int f = f_lo; f <= f_hi; f++) {
                        const unsigned int base = f * frame_units;
                        if (!MULTI || (gu >= base && gu - base < frame_units)) {
                            const unsigned int lu = gu - base;
                            const int pixel = unit_to_pixel(til, lu >> batch_log2);
                            const int32_t hseed = hash_pt(first_pass + (int)(lu & ((1u << batch_log2) - 1u)));
                            const DevCamera cam = MULTI ? load_const(out.cams + f) : load_const(&P->cam);
                            PathState g;
                            generate_path(cam, cfg, pixel, hseed, &g);
                            gen_ring_put(ring, PT_LANE, g, path_seed(hseed, pixel), gu);
                        }
                    }
                }
                cursor.cur = cursor.end;
                __builtin_amdgcn_wave_barrier();  // the ring's writes before the lanes read it (one wave: in order)
                const int rest = taken - avail;
                if (want && !got && rank - avail < n) {
                    gen_ring_get(ring, rank - avail, ps, pseed, u);
                    got = true;
                }
                ring_head = rest < n ? rest : n;
                ring_end = n;
            } else {
                ring_head = ring_end;
                drained = true;
            }
            if (PROF && drained && t_drain == 0) t_drain = __builtin_amdgcn_s_memrealtime();
            if (want) {
                if (got) {
                    lds_unit[PT_TID] = u;
                    depth = 0;
                    if (cfg.max_depth > 0) {
                        mode = LANE_NEW;
                    } else {
                        finish_unit(til, cfg, out, ps, u, MULTI ? frame_units : 0u, first_pass,
                                    write_u8, batch_log2, (float)cfg.max_depth * 2.0f, depth);
                    }
                } else if (drained) {
                    mode = LANE_DONE;
                }
            }
        }
        if (mode == LANE_NEW) {
            if (FEAT & PT_FEAT_MBOUND) {
                wbound = medium_bound(sc, cfg, ps.medium, depth, pseed);
                mode = begin_segment(sc, roots, lds_mesh, lds_root, ps, inv, h, w, mesh, wbound);
            } else {
                mode = begin_segment(sc, roots, lds_mesh, lds_root, ps, inv, h, w, mesh);
            }
        }
        if (!__any(mode != LANE_DONE)) break;
        if (PROF) { const unsigned long long t = __builtin_readcyclecounter(); prof[8] += t - tc; tc = t; }

        const unsigned long long ready = __ballot(mode == LANE_READY);
        const unsigned long long walking = __ballot(mode == LANE_WALK) | __ballot(mode == LANE_TRI);
        if (ready && (__popcll(walking) <= (unsigned int)walk_min || __popcll(ready) >= (unsigned int)shade_min)) {
            if (PROF) { prof[3]++; prof[4] += (unsigned long long)__popcll(ready); }
            if (PROF && drained) tail_segments += (unsigned long long)__popcll(ready);
            segments += (unsigned long long)__popcll(ready);
            bool alive = false;
            if (mode == LANE_READY) {
                // the rest of trace_ray_kernel for this segment (:456-624)
                alive = shade_hit<false, FEAT>(sc, cfg, depth, pseed, &ps, h, &none, nullptr);
            }
            if (PROF) tc2 = __builtin_readcyclecounter();
            if (mode == LANE_READY) {  // the pass's end for this unit, or the next trace step
                depth++;
                if (!alive || depth >= cfg.max_depth) {
                    const unsigned int un = lds_unit[PT_TID];
                    finish_unit(til, cfg, out, ps, un, MULTI ? frame_units : 0u, first_pass, write_u8, batch_log2, (float)cfg.max_depth * 2.0f, depth);
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
        // closest_hit's merge of a finished mesh walk (:443-454), then the next mesh or READY
        auto mesh_done = [&]() {
            if (w.tri >= 0 && w.t < h.t) {
                h.t = w.t; h.t1 = w.t1; h.t2 = w.t2; h.prim = w.tri; h.type = 2;
            }
            bool more;
            int2 range = make_int2(0, 0);
            if (roots) {
                more = next_root_mesh(lds_mesh, lds_root, mesh, range);
            } else {
                mesh++;
                if (sc.mesh_num <= PT_LDS_MESHES) more = start_mesh_next(lds_next, mesh, range);
                else more = start_mesh(sc, lds_mesh, mesh, range);
            }
            // the walk state is reset whether or not a mesh is left (a READY lane does not read it), so
            // the branches above only produce a range and the compiler merges no walk fields
            walk_start(w, range, (FEAT & PT_FEAT_MBOUND) ? wbound : __builtin_inff());
            mode = more ? LANE_WALK : LANE_READY;
        };
        // the parked triangle's geometry, loaded at the park; scoped to the walk loop, which no lane leaves
        // parked (the last step flushes the batch), so it is not live across shading
        float4 pta = make_float4(0.0f, 0.0f, 0.0f, 0.0f), ptb = pta, ptc = pta;
        for (int k = 0; k < walk_steps; k++) {
            // two ballots, not one of (WALK || TRI): the compiler materialises an OR'ed predicate as a 0/1 VGPR
            // and compares it again (two VALU more per step)
            if (k > 0 && (__ballot(mode == LANE_WALK) | __ballot(mode == LANE_TRI)) == 0ull) break;
            if (PROF) {
                prof[1]++; prof[2] += (unsigned long long)__popcll(__ballot(mode == LANE_WALK));
                prof[12] += (unsigned long long)__popcll(__ballot(mode == LANE_TRI));
                if (drained) prof[11] += 1ull | ((unsigned long long)__popcll(__ballot(mode == LANE_WALK)) << 32);
                prof[13] += (unsigned long long)__popcll(__ballot(mode == LANE_READY));
                prof[14] += (unsigned long long)__popcll(__ballot(mode == LANE_WANT || mode == LANE_DONE));
            }
            if (mode == LANE_WALK) {
                // a leaf whose box passes: the lane parks with its triangle, which came with the step's records
                if (PT_WALK_PRIO) __builtin_amdgcn_s_setprio(PT_WALK_PRIO);  // until the step's loads issue (pt_path.h)
                if (walk_box_inline(rn, ps.o, inv, w, ptri, pta, ptb, ptc)) mode = LANE_TRI;
            }
            // leaf triangles are tested in batches of at least tri_min lanes (or when no lane can walk on,
            // or on the round's last step, so that no lane leaves the walk loop parked): the triangle test
            // then runs with many lanes active instead of one or two
            const unsigned long long pend = __ballot(mode == LANE_TRI);
            if (pend && (__popcll(pend) >= (unsigned int)tri_min || !__any(mode == LANE_WALK) || k == walk_steps - 1)) {
                if (PROF) { prof[5]++; prof[6] += (unsigned long long)__popcll(pend); }
                if (mode == LANE_TRI) {
                    walk_tri_geom(pta, ptb, ptc, ps.o, ps.d, w, ptri);
                    w.pos++;  // past the leaf's triangle record too
                    mode = LANE_WALK;
                }
            }
            // a lane whose mesh walk ended in this step (after a box or after its triangle) merges it and
            // starts the next mesh: one mesh_done site for both
            if (mode == LANE_WALK && w.pos == w.end) mesh_done();
        }
        if (PROF) prof[10] += __builtin_readcyclecounter() - tc;
    }

    if (PT_LANE == 0) {
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
            atomicAdd(&tl[10], gen_batches); atomicAdd(&tl[11], live_lane_rounds);
        }
    }
#undef PT_LANE
#undef PT_TID
}

// The running sum over a batch of passes, in pass order (path_tracer_kernel.cu:644-651 applied
// pass after pass), then the 8-bit output of the batch's last pass.
// frame: which frame copy of a pt_render_frames launch (0 otherwise)
// frame's running sum `image` and 8-bit output `image256` (the launch's own, or a pt_render_frames frame's)
__device__ __forceinline__ void accumulate_unit(const LaunchParams* __restrict__ P, int first_pass, int batch_log2,
                                                int write_u8, int frame, unsigned int lu, float* __restrict__ image,
                                                uint8_t* __restrict__ image256) {
    const int pixel = unit_to_pixel(P->til, lu);
    const int batch = 1 << batch_log2;
    float* img = image + (size_t)pixel * 3;
    const float* pr = P->out.pass_rad + (((size_t)frame * (size_t)P->til.unit_count + lu) << batch_log2) * 3;
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
    if (write_u8 && image256) store_u8(P->cfg, sum, first_pass + batch - 1, image256 + (size_t)pixel * 3);
}

__global__ __launch_bounds__(PT_BLOCK) void accumulate_kernel(const LaunchParams* __restrict__ P, int first_pass,
                                                              int batch_log2, int write_u8, int frame,
                                                              float* __restrict__ image, uint8_t* __restrict__ image256) {
    const unsigned int lu = blockIdx.x * PT_BLOCK + threadIdx.x;
    if (lu >= (unsigned int)P->til.unit_count) return;
    accumulate_unit(P, first_pass, batch_log2, write_u8, frame, lu, image, image256);
}

// Every frame of a pt_render_frames launch in one launch (blockIdx.y = frame): frame f's running sum and 8-bit
// output are images[f] and images256[f] of a device table of 2 x frames pointers (images256[f] may be null).
__global__ __launch_bounds__(PT_BLOCK) void accumulate_frames_kernel(const LaunchParams* __restrict__ P, int first_pass,
                                                                     int batch_log2, int write_u8, int frames,
                                                                     const uint64_t* __restrict__ ptrs) {
    const unsigned int lu = blockIdx.x * PT_BLOCK + threadIdx.x;
    if (lu >= (unsigned int)P->til.unit_count) return;
    const int f = (int)blockIdx.y;
    float* image = reinterpret_cast<float*>(ptrs[f]);
    uint8_t* image256 = reinterpret_cast<uint8_t*>(ptrs[frames + f]);
    accumulate_unit(P, first_pass, batch_log2, write_u8, f, lu, image, image256);
}

// One pass of a batched launch added into the running sum: pass `pass` is slot j of every unit's run of
// 2^batch_log2 pass radiances in rad (path_tracer_kernel.cu:644-651 for that pass), then its 8-bit output.
// The reference ABI's pass cache (pt_runtime.cpp abi_render_pass) serves one pass per call this way.
// src: the running sum the pass adds into (null: the image itself, in place); the reference ABI keeps the
// caller's uploaded sum apart so that a call can be redone (pt_runtime.cpp path_tracer_kernel).
__global__ __launch_bounds__(PT_BLOCK) void accumulate_one_kernel(const LaunchParams* __restrict__ P, int pass,
                                                                  int batch_log2, int j, int write_u8,
                                                                  const float* __restrict__ rad, const float* src,
                                                                  int unit_begin, int unit_end) {
    const unsigned int lu = unit_begin + blockIdx.x * PT_BLOCK + threadIdx.x;
    if (lu >= (unsigned int)unit_end) return;
    const int pixel = unit_to_pixel(P->til, lu);
    float* img = P->out.image + (size_t)pixel * 3;
    const float* old = (src ? src : P->out.image) + (size_t)pixel * 3;
    const float* pr = rad + (((size_t)lu << batch_log2) + (size_t)j) * 3;
    const v3 c = mk3(pr[0], pr[1], pr[2]);
    const v3 sum = pass == 1 ? c : mk3(old[0], old[1], old[2]) + c;
    img[0] = sum.x; img[1] = sum.y; img[2] = sum.z;
    if (write_u8 && P->out.image256) store_u8(P->cfg, sum, pass, P->out.image256 + (size_t)pixel * 3);
}

hipError_t launch_accumulate_one(const LaunchParams* params_dev, int unit_begin, int unit_end, int pass, int batch_log2,
                                 int j, int write_u8, const float* rad, const float* src, hipStream_t stream) {
    const int units = unit_end - unit_begin;
    if (units <= 0) return hipSuccess;
    hipLaunchKernelGGL(accumulate_one_kernel, dim3((units + PT_BLOCK - 1) / PT_BLOCK), dim3(PT_BLOCK), 0, stream,
                       params_dev, pass, batch_log2, j, write_u8, rad, src, unit_begin, unit_end);
    return hipGetLastError();
}

// An order-independent 64-bit digest of words [begin, end) of a buffer, added into *out: the sum over words of
// splitmix64((index << 32) | word) (wrapping). The reference ABI digests the running sum it returns and the one the
// caller hands back, so it can tell that passes ran elsewhere in between (pt_runtime.cpp path_tracer_kernel).
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// One non-returning atomic per workgroup into ONE word: a word takes ~88 atomics per us (pt_work.h), so the grid is
// kept to 256 workgroups (the sum is order-free). With one atomic per wave over 2048 workgroups, the eight digest
// launches of a reference-ABI call spent ~0.7 ms queued on that word (1.55 instead of ~0.9 ms per continuation call).
#define PT_DIGEST_BLOCKS 256
__global__ __launch_bounds__(PT_BLOCK) void digest_words_kernel(const uint32_t* __restrict__ p, unsigned long long begin,
                                                                unsigned long long end, unsigned long long* out) {
    __shared__ unsigned long long part[PT_BLOCK / 64];
    unsigned long long h = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * PT_BLOCK;
    for (unsigned long long i = begin + blockIdx.x * PT_BLOCK + threadIdx.x; i < end; i += stride)
        h += splitmix64((i << 32) | p[i]);
    for (int off = 32; off > 0; off >>= 1) h += __shfl_xor(h, off);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int w = 0; w < PT_BLOCK / 64; w++) s += part[w];
        atomicAdd(out, s);
    }
}

hipError_t launch_digest_words(const void* p, size_t begin, size_t end, unsigned long long* out, hipStream_t stream) {
    if (end <= begin) return hipSuccess;
    const size_t blocks = std::min<size_t>((end - begin + PT_BLOCK - 1) / PT_BLOCK, PT_DIGEST_BLOCKS);
    hipLaunchKernelGGL(digest_words_kernel, dim3((unsigned)blocks), dim3(PT_BLOCK), 0, stream,
                       static_cast<const uint32_t*>(p), (unsigned long long)begin, (unsigned long long)end, out);
    return hipGetLastError();
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
    m.ratio_front = air_n / m.refraction_index;
    m.ratio_back = m.refraction_index / air_n;
    m.tir_front = asin_pt(m.ratio_back);
    m.tir_back = asin_pt(m.ratio_front);
    // the zero-specular shortcut (shade_hit): a zero specular colour, and a GGX alpha for which the shadow term is
    // finite on (near-)unit vectors (alpha^2 normal and > 0, alpha <= 4). alpha == 0 (roughness 0) is excluded:
    // ggx_g1 is 2 / (1 + sqrt(1 + 0 * inf)) = NaN when (v.n)^2 underflows, and the reference keeps that path.
    m.spec_zero = m.specular[0] == 0.0f && m.specular[1] == 0.0f && m.specular[2] == 0.0f &&
                  m.rough_alpha >= 0x1p-60f && m.rough_alpha <= 4.0f;
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
        case 11: r0 = sqrt_exact(a); r1 = sqrtf(a); break;
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

// pass_kernel: the instrumented (STATS) kernel that feeds the roofline model, the leaf-size > 1 path and
// the PT_UNIFIED=0 fallback.
static PassFn pass_fn(bool leaf1, bool stats, int minw) {
    if (leaf1 && !stats) {
        if (minw == 4) return pass_kernel<true, false, 4>;
        if (minw == 6) return pass_kernel<true, false, 6>;
        if (minw == 7) return pass_kernel<true, false, 7>;
        if (minw == 8) return pass_kernel<true, false, 8>;
        return pass_kernel<true, false, 5>;
    }
    if (leaf1 && stats) return pass_kernel<true, true, 5>;
    if (!stats) return pass_kernel<false, false, 5>;
    return pass_kernel<false, true, 5>;
}

// PT_MIN_WAVES overrides the occupancy target: 8 waves/SIMD for pass_kernel (64 VGPRs); for pass_kernel_u
// 8 when the scene reaches neither textures nor a participating medium (64 VGPRs without spills since round 4
// recomputes the hit point and the clamp bound where they are used: metric +1.6 % with frame groups, +1.2 %
// without, C3 +1.1 %, C2 +0.9 %; profiles/r04/knobs/waves_ab2.txt), 7 with textures (72 VGPRs, one cold
// spill; +6.7 % over 6 on C5) and 7 with a medium, exact or bounded (72 VGPRs, no spills; round 4 on the reference
// tree chose 6: C4 5567-5573 vs 5709-5731 Mrays/s at 7, profiles/r04/knobs/waves_ab1.txt; round 6 on the SAH
// tree, with 22 % fewer L2 requests, 7 wins: C4 8138-8149 vs 7975-7983, C4 bounded 12275-12294 vs 11489-11523,
// profiles/r06/knobs/c4_waves.txt).
int pass_min_waves(bool unified, int feat, bool small) {
    static int w = [] {
        const char* e = getenv("PT_MIN_WAVES");
        int v = e ? atoi(e) : 0;
        return (v >= 5 && v <= 8) ? v : 0;
    }();
    if (w) return w;
    if (!unified) return 8;
    // 8 without textures or media (64 VGPRs, no spills since the hit point is recomputed at use: metric +0.8 %
    // one frame per launch, C3 +1 %); 7 with a medium (above; the bounded walk's instances exist at 6 and 7)
    static const int plain = env_int("PT_PLAIN_WAVES", 8, 5, 8);
    static const int medium = env_int("PT_MEDIUM_WAVES", 7, 5, 8);
    // textures: 8 since round 6 (64 VGPRs with 5 cold spills, 16 B of scratch; C5 9876-9881 vs 9779-9785 Mrays/s at 7,
    // profiles/r06/knobs/c5_waves.txt; round 4's 7 over 6 was +6.7 %)
    static const int tex = env_int("PT_TEX_WAVES", 8, 5, 8);
    // a small launch (C1's 512x512x4 units: 128 per wave at 8 waves) is mostly its waves' first chunks and
    // tails: 7 waves (C1 33129-34058 vs 30978-31236 Mrays/s at 8, profiles/r04/knobs/c1_waves.txt)
    return (feat & PT_FEAT_MBOUND) ? (medium >= 7 ? 7 : 6) : (feat & PT_FEAT_MEDIUM) ? medium
                                   : small ? std::min((feat & PT_FEAT_TEX) ? tex : plain, 7) : (feat & PT_FEAT_TEX) ? tex : plain;
}

// PT_UNIFIED=0 selects pass_kernel for the default configuration (leaf size 1, uninstrumented);
// otherwise pass_kernel_u runs it. PT_SHADE_MIN / PT_WALK_STEPS tune pass_kernel_u.
bool unified_enabled() {
    static const int on = env_int("PT_UNIFIED", 1, 0, 1);
    return on != 0;
}

using PassFnU = void (*)(const LaunchParams*, int, int, int, int, int, int, int, int);

// pass_kernel_u specialised on the scene's features (pt_path.h PT_FEAT_*): feat is what the scene can reach;
// PT_FEAT_SPECIALISE=0 keeps the all-features kernel. `feat_used` receives the instance's features, so the
// kernel description names the kernel that runs. PT_UPROF=1: the profiling instance (6 waves, all features).
// multi: the MULTI instance (pt_render_frames) for pass_min_waves' choice: 8 or 7 waves without textures or
// media, 7 with textures, 6 with a medium (the instances built; PT_UPROF does not apply to it). pass_grid_size
// sizes the grid from the same instance.
static PassFnU pass_fn_u(int minw, int feat, bool multi, int* feat_used, int* minw_used) {
    static const int spec = env_int("PT_FEAT_SPECIALISE", 1, 0, 1);
    static const int prof = env_int("PT_UPROF", 0, 0, 1);
    if (!spec) feat = PT_FEAT_ALL | (feat & PT_FEAT_MBOUND);
    if (multi) {  // render_frames fuses frames only without the medium bound
        feat &= PT_FEAT_ALL;
        *feat_used = feat;
        *minw_used = (feat & PT_FEAT_MEDIUM) ? 6 : 7;
        if (feat == 0 && minw >= 8) { *minw_used = 8; return pass_kernel_u<8, false, 0, true>; }
        switch (feat) {
            case 0: return pass_kernel_u<7, false, 0, true>;
            case 1: return pass_kernel_u<6, false, 1, true>;
            case 2: return pass_kernel_u<7, false, 2, true>;
            default: return pass_kernel_u<6, false, 3, true>;
        }
    }
    if (prof) { *feat_used = PT_FEAT_ALL; *minw_used = 6; return pass_kernel_u<6, true, PT_FEAT_ALL>; }
    *feat_used = feat;
    *minw_used = minw;
#define PT_U_CASE(W, F) case W * 8 + F: return pass_kernel_u<W, false, F>;
    switch (minw * 8 + feat) {
        PT_U_CASE(5, 0) PT_U_CASE(5, 1) PT_U_CASE(5, 2) PT_U_CASE(5, 3)
        PT_U_CASE(6, 0) PT_U_CASE(6, 1) PT_U_CASE(6, 2) PT_U_CASE(6, 3) PT_U_CASE(6, 5) PT_U_CASE(6, 7)
        PT_U_CASE(7, 0) PT_U_CASE(7, 1) PT_U_CASE(7, 2) PT_U_CASE(7, 3) PT_U_CASE(7, 5) PT_U_CASE(7, 7)
        PT_U_CASE(8, 0) PT_U_CASE(8, 1) PT_U_CASE(8, 2) PT_U_CASE(8, 3)
        default: break;
    }
#undef PT_U_CASE
    *feat_used = PT_FEAT_ALL | (feat & PT_FEAT_MBOUND);
    *minw_used = 6;
    if (feat & PT_FEAT_MBOUND) return pass_kernel_u<6, false, PT_FEAT_ALL | PT_FEAT_MBOUND>;
    return pass_kernel_u<6, false, PT_FEAT_ALL>;
}

// pass_kernel_u keeps every material and sphere in LDS: scenes whose tables exceed PT_LDS_TABLES bytes
// (about 256 materials and 256 spheres) run pass_kernel.
#define PT_LDS_TABLES (32 * 1024)
// pass_kernel_u walks the inline-leaf layout only (walk_box_inline): without it (leaf size > 1, or a leaf whose
// skip index is not the next record) the launch runs pass_kernel, which follows every node's own skip index
static bool use_unified(const PassChoice& pc, int lds_bytes) {
    return pc.leaf1 && pc.il && !pc.stats && unified_enabled() && lds_bytes <= PT_LDS_TABLES;
}

bool pass_uses_unified(const PassChoice& pc, int lds_bytes) { return use_unified(pc, lds_bytes); }

// The inline-leaf copy of the node array that pass_kernel_u walks (pt_path.h walk_box_inline): record k of
// `nodes` goes to record np[k] of `out`; a leaf (slot >= 0, one triangle per leaf) takes two records,
// its box with e2.z in the free skip word and then its triangle from tri_geom; an internal record keeps
// its box with the skip index remapped through np (np[R] is the end of the last mesh).
__global__ void inline_leaves_kernel(const float4* __restrict__ nodes, const float4* __restrict__ tri_geom,
                                     const int* __restrict__ np, int R, float4* __restrict__ out) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= R) return;
    const float4 lo = nodes[2 * k], hi = nodes[2 * k + 1];
    const int slot = f2i(hi.w), p = np[k];
    if (slot >= 0) {
        const float4 a = tri_geom[3 * slot], e1 = tri_geom[3 * slot + 1], e2 = tri_geom[3 * slot + 2];
        out[2 * p] = make_float4(lo.x, lo.y, lo.z, e2.z);
        out[2 * p + 1] = hi;
        out[2 * p + 2] = make_float4(a.x, a.y, a.z, e1.x);
        out[2 * p + 3] = make_float4(e1.y, e1.z, e2.x, e2.y);
    } else {
        out[2 * p] = make_float4(lo.x, lo.y, lo.z, __int_as_float(np[f2i(lo.w)]));
        out[2 * p + 1] = hi;
    }
}

__global__ __launch_bounds__(PT_BLOCK) void cube_float_kernel(const uint8_t* __restrict__ cube, int texels,
                                                              float4* __restrict__ out) {
    const int i = blockIdx.x * PT_BLOCK + threadIdx.x;
    if (i >= texels) return;
    const unsigned int t = texel_raw(cube, i);
    out[i] = make_float4(texel_c(t, 0), texel_c(t, 1), texel_c(t, 2), 0.0f);
}

hipError_t launch_cube_float(const uint8_t* cube, int texels, float4* out, hipStream_t stream) {
    if (texels <= 0) return hipSuccess;
    hipLaunchKernelGGL(cube_float_kernel, dim3((texels + PT_BLOCK - 1) / PT_BLOCK), dim3(PT_BLOCK), 0, stream, cube,
                       texels, out);
    return hipGetLastError();
}

hipError_t launch_inline_leaves(const float4* nodes, const float4* tri_geom, const int* np, int R, float4* out,
                                hipStream_t stream) {
    if (R <= 0) return hipSuccess;
    hipLaunchKernelGGL(inline_leaves_kernel, dim3((R + 255) / 256), dim3(256), 0, stream, nodes, tri_geom, np, R, out);
    return hipGetLastError();
}

hipError_t launch_pass(const LaunchParams* params_dev, const PassChoice& pc, int first_pass, int batch_log2,
                       int write_u8, int grid, int lds_bytes, hipStream_t stream) {
    if (use_unified(pc, lds_bytes)) {
        // 64-unit chunks, a 28-lane shading batch, 7 walk steps per round, triangle batches of 4 lanes:
        // measured best with frames in flight (7 steps since the end of round 3: metric
        // +0.4 %, C3 +0.9 %, C4/C5 +0.1-0.3 %, profiles/r03/walk_steps/; 4 parked lanes instead of 6 since the
        // fused multiply-adds made the triangle test cheaper: +0.3 % over four rounds, profiles/r04/knobs/)
        // (the generation ring holds one chunk: 1..64 units)
        static const int chunk = env_int("PT_CHUNK_MEGA", 64, 1, PT_RING);
        // the shading batch waits for 32 ready lanes with a medium walked exactly (the medium step makes a batch
        // dearer; round 4 on the reference tree: 40, C4 5952-5966 vs 5747 Mrays/s at 28, profiles/r04/knobs/
        // c4_c5_shade_min.txt; round 6 on the SAH tree, whose walks are shorter: 32 7955-7975 vs 7813-7839 at 40,
        // 24 / 28 / 36 7876-7954, 48 7134-7150, profiles/r06/knobs/c4_shade_min.txt), 28 otherwise (C5 at 32 / 36:
        // ±0 / -1 %; the medium-bounded walk, shorter: 9450 at 40 vs 9573-9597)
        static const int shade_env = env_int("PT_SHADE_MIN", 0, 0, 64);
        const bool dear = (pc.feat & PT_FEAT_MEDIUM) && !(pc.feat & PT_FEAT_MBOUND);
        const int shade_min = shade_env ? shade_env : dear ? 32 : 28;
        static const int walk_steps = env_int("PT_WALK_STEPS", 7, 1, 64);
        static const int tri_min = env_int("PT_TRI_MIN", 4, 1, 64);
        static const int walk_min = env_int("PT_WALK_MIN", 8, 0, 64);
        int fu, wu;
        const PassFnU fn = pass_fn_u(pass_min_waves(true, pc.feat, pc.small), pc.feat, pc.multi, &fu, &wu);
        const LaunchParams* a0 = params_dev;
        int a1 = first_pass, a2 = write_u8, a3 = chunk, a4 = batch_log2, a5 = shade_min, a6 = walk_steps, a7 = tri_min,
            a8 = walk_min;
        void* args[] = {&a0, &a1, &a2, &a3, &a4, &a5, &a6, &a7, &a8};
        hipError_t e = hipLaunchKernel((const void*)fn, dim3(grid), dim3(PT_UBLOCK), args, (size_t)lds_bytes, stream);
        if (e != hipSuccess) return e;
        return hipGetLastError();
    }
    PassFn fn = pass_fn(pc.leaf1, pc.stats, pass_min_waves(false, pc.feat, pc.small));
    const LaunchParams* a0 = params_dev;
    static const int chunk = env_int("PT_CHUNK_MEGA", 32, 0, 4096);
    int a1 = first_pass, a2 = write_u8, a3 = chunk, a4 = batch_log2;
    void* args[] = {&a0, &a1, &a2, &a3, &a4};
    hipError_t e = hipLaunchKernel((const void*)fn, dim3(grid), dim3(PT_BLOCK), args, 0, stream);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t launch_accumulate(const LaunchParams* params_dev, int units, int first_pass, int batch_log2, int write_u8,
                             hipStream_t stream, int frame, float* image, uint8_t* image256) {
    if (units <= 0) return hipSuccess;
    hipLaunchKernelGGL(accumulate_kernel, dim3((units + PT_BLOCK - 1) / PT_BLOCK), dim3(PT_BLOCK), 0, stream,
                       params_dev, first_pass, batch_log2, write_u8, frame, image, image256);
    return hipGetLastError();
}

hipError_t launch_accumulate_frames(const LaunchParams* params_dev, int units, int first_pass, int batch_log2,
                                    int write_u8, int frames, const uint64_t* ptrs_dev, hipStream_t stream) {
    if (units <= 0 || frames <= 0) return hipSuccess;
    if (frames > 65535) return hipErrorInvalidValue;  // gridDim.y
    hipLaunchKernelGGL(accumulate_frames_kernel, dim3((units + PT_BLOCK - 1) / PT_BLOCK, frames), dim3(PT_BLOCK), 0,
                       stream, params_dev, first_pass, batch_log2, write_u8, frames, ptrs_dev);
    return hipGetLastError();
}

hipError_t launch_u8(const DevConfig& cfg, const float* image, uint8_t* image256, int pixel_count, int pass,
                     hipStream_t stream) {
    if (pixel_count <= 0) return hipSuccess;
    int grid = (pixel_count + PT_BLOCK - 1) / PT_BLOCK;
    hipLaunchKernelGGL(u8_kernel, dim3(grid), dim3(PT_BLOCK), 0, stream, cfg, image, image256, pixel_count, pass);
    return hipGetLastError();
}

// The pass kernel launch_pass picks for these arguments, as text (bench.py's roofline.kernel): derived
// from the instance pass_fn_u actually selects.
std::string pass_kernel_desc(const PassChoice& pc, int lds_bytes) {
    char buf[160];
    if (use_unified(pc, lds_bytes)) {
        int fu, wu;
        (void)pass_fn_u(pass_min_waves(true, pc.feat, pc.small), pc.feat, pc.multi, &fu, &wu);
        static const int prof = env_int("PT_UPROF", 0, 0, 1);
        std::snprintf(buf, sizeof(buf), "pass_kernel_u<MINW=%d,FEAT=%d%s>", wu, fu,
                      pc.multi ? ",MULTI" : prof ? ",PROF" : "");
    } else {
        std::snprintf(buf, sizeof(buf), "pass_kernel<LEAF1=%d,STATS=%d,MINW=%d>", pc.leaf1 ? 1 : 0, pc.stats ? 1 : 0,
                      pass_min_waves(false, pc.feat, pc.small));
    }
    return buf;
}

int pass_grid_size(const PassChoice& pc, int lds_bytes) {
    int dev = 0, cus = 0, blocks = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    const bool u = use_unified(pc, lds_bytes);
    int fu, wu;
    const void* fn = u ? (const void*)pass_fn_u(pass_min_waves(true, pc.feat, pc.small), pc.feat, pc.multi, &fu, &wu)
                       : (const void*)pass_fn(pc.leaf1, pc.stats, pass_min_waves(false, pc.feat, pc.small));
    const size_t lds = u ? (size_t)lds_bytes : 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, u ? PT_UBLOCK : PT_BLOCK, lds) != hipSuccess || blocks <= 0)
        blocks = u ? 4 * PT_BLOCK / PT_UBLOCK : 4;
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
