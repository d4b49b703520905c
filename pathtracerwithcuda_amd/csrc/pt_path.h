// pt_path.h — per-ray device functions of the radiance loop.
//
// Each function restates one reference function (file:line given); the operation order of
// every float expression follows the reference source, and the fused multiply-adds of the
// reference's CUDA build (nvcc -fmad=true) are written out as fmaf at the sites its contraction
// rule gives (pt_math.h header), the rest compiled with contraction off, so the
// result is reproducible on the host (oracle/) bit-for-bit.
#pragma once

#include "pt_math.h"
#include "pt_scene.h"

namespace pt {

#if defined(__HIP_DEVICE_COMPILE__)
#define PT_LDG(p) __builtin_nontemporal_load(p)
#endif

__device__ __forceinline__ v3 f4xyz(float4 a) { return mk3(a.x, a.y, a.z); }

// Whole-record loads. Left alone, the compiler narrows a float4 load to the components used before
// the next branch (dwordx3 for a box, then a dependent dword for next/slot after the test), which
// puts a second L2 round trip on every node. The empty asm makes all four lanes live at once, so
// each record is one global_load_dwordx4 and all loads of a record are in flight together.
__device__ __forceinline__ float4 ld_record(const float4* p) {
    float4 v = *p;
    asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
    return v;
}
__device__ __forceinline__ int f2i(float f) { return __float_as_int(f); }

// Scene records through buffer descriptors: a raw_buffer_load_b128 is never narrowed by the
// compiler and is only waited for at its first use, so a load can be issued early (prefetch).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Wave-uniform copies of scene pointers and sizes. Inside the divergent path loop the compiler can
// lose track of their uniformity and keep them in VGPRs; a buffer descriptor held in VGPRs turns
// every buffer load into a waterfall loop (readfirstlane x4, compare, exec juggling per load). The
// scene is the same for every lane, so readfirstlane is exact and pins them to SGPRs.
__device__ __forceinline__ int uniform_int(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned int lo = (unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)v);
    const unsigned int hi = (unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)(v >> 32));
    return (T*)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(uniform_ptr(base)), (short)0, uniform_int(bytes),
                                             0x00020000);
}
__device__ __forceinline__ float4 bload(__amdgpu_buffer_rsrc_t r, int byte_offset) {
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_offset, 0, 0);
    float4 f;
    f.x = __uint_as_float(v.x); f.y = __uint_as_float(v.y); f.z = __uint_as_float(v.z); f.w = __uint_as_float(v.w);
    return f;
}

// path_tracer_kernel.cu:46-52: in - (2 dot) n, the product fused into the subtraction
__device__ __forceinline__ v3 reflection(v3 n, v3 in) {
    const float s = -(2.0f * dot(n, in));
    return fma3(n, s, in);
}

// path_tracer_kernel.cu:54-83; ratio = in_n / out_n (a per-material constant, DevMaterial::ratio_front /
// ratio_back, computed by material_consts_kernel with the same division)
__device__ __forceinline__ v3 refraction(v3 n, v3 in, float ratio) {
    v3 i = in * -1.0f;
    float ndi = dot(n, i);
    float a = ratio * ndi;
    // 1 - (r r)(1 - ndi ndi), both subtractions of a product contracted
    float b = fmaf(-(ratio * ratio), fmaf(-ndi, ndi, 1.0f), 1.0f);
    if (b < 0.0f) return mk3(0.0f, 0.0f, 0.0f);
    // n (a -+ sqrt b) - r i: the left product fused
    const float q = ndi > 0 ? a - sqrt_pt(b) : a + sqrt_pt(b);
    return mk3(fmaf(n.x, q, -(ratio * i.x)), fmaf(n.y, q, -(ratio * i.y)), fmaf(n.z, q, -(ratio * i.z)));
}

// Orthonormal frame of sample_on_hemisphere_* (path_tracer_kernel.cu:175-189). The reference
// leaves any_direction uninitialised when no component is below 1/sqrt(3); that cannot happen
// for |n| <= 1, and (0,0,1) keeps the impossible case defined.
__device__ __forceinline__ void tangent_frame(v3 n, v3* vi, v3* vj) {
    v3 any;
    if (fabsf(n.x) < kSQRT_ONE_THIRD) any = mk3(1.0f, 0.0f, 0.0f);
    else if (fabsf(n.y) < kSQRT_ONE_THIRD) any = mk3(0.0f, 1.0f, 0.0f);
    else any = mk3(0.0f, 0.0f, 1.0f);
    *vi = normalize(cross(n, any));
    *vj = cross(n, *vi);
}

// cos_theta n + (cos phi sin_theta) vi + (sin phi sin_theta) vj (path_tracer_kernel.cu:191,222), contracted:
// ((ct n + c vi) + s vj) -> fmaf(s, vj, fmaf(ct, n, c vi))
__device__ __forceinline__ v3 hemisphere_combine(v3 n, float cos_theta, float c, v3 vi, float s, v3 vj) {
    return fma3(vj, s, fma3(n, cos_theta, vi * c));
}

// The common tail of sample_on_hemisphere_cosine_weight / _ggx_weight (path_tracer_kernel.cu:174-191):
// the tangent frame of n and the direction at (theta, phi = 2 pi r2).
__device__ __forceinline__ v3 hemisphere_dir(v3 n, float cos_theta, float sin_theta, float r2) {
    float phi = r2 * kTWO_PI;
    v3 vi, vj;
    tangent_frame(n, &vi, &vj);
    float sp, cp;
    sincos_pt(phi, &sp, &cp);
    return hemisphere_combine(n, cos_theta, cp * sin_theta, vi, sp * sin_theta, vj);
}

// path_tracer_kernel.cu:163-192
__device__ __forceinline__ v3 sample_cosine(v3 n, float r1, float r2) {
    float cos_theta = sqrt_pt(r1);
    float sin_theta = sqrt_pt(fmaf(-cos_theta, cos_theta, 1.0f));
    float phi = r2 * kTWO_PI;
    v3 vi, vj;
    tangent_frame(n, &vi, &vj);
    float sp, cp;
    sincos_pt(phi, &sp, &cp);
    return hemisphere_combine(n, cos_theta, cp * sin_theta, vi, sp * sin_theta, vj);
}

// path_tracer_kernel.cu:194-223
__device__ __forceinline__ v3 sample_ggx(v3 n, float roughness, float r1, float r2) {
    float theta = atan_pt(roughness * sqrt_pt(r1) / sqrt_pt(1.0f - r1));
    float phi = r2 * kTWO_PI;
    float sin_theta, cos_theta;
    sincos_pt(theta, &sin_theta, &cos_theta);
    v3 vi, vj;
    tangent_frame(n, &vi, &vj);
    float sp, cp;
    sincos_pt(phi, &sp, &cp);
    return hemisphere_combine(n, cos_theta, cp * sin_theta, vi, sp * sin_theta, vj);
}

// path_tracer_kernel.cu:225-236
__device__ __forceinline__ v3 sample_sphere(float r1, float r2) {
    float cos_theta = fmaf(r1, 2.0f, -1.0f);
    float sin_theta = sqrt_pt(fmaf(-cos_theta, cos_theta, 1.0f));
    float phi = r2 * kTWO_PI;
    float sp, cp;
    sincos_pt(phi, &sp, &cp);
    return mk3(cos_theta, cp * sin_theta, sp * sin_theta);
}

// path_tracer_kernel.cu:238-249 (__powf(E, -a*d) -> exp)
__device__ __forceinline__ v3 absorption(const float a[3], float d) {
    return mk3(exp_pt(-1.0f * a[0] * d), exp_pt(-1.0f * a[1] * d), exp_pt(-1.0f * a[2] * d));
}

// path_tracer_kernel.cu:251-273
__device__ __forceinline__ float ggx_g1(float roughness, v3 macro, v3 micro, v3 dir) {
    v3 v = -1.0f * dir;
    float vdn = dot(v, macro);
    float vdm = dot(v, micro);
    // (vdm / vdn) > 0 without the division where its outcome is the operands' signs: for
    // |vdm| >= 2^-100 and |vdn| <= 2^40 the quotient is neither NaN nor rounded to 0, and its sign is
    // the XOR of the sign bits (a signed zero vdn included: x / +-0 = +-inf). Elsewhere, the division.
    bool positive;
    if (fabsf(vdm) >= 0x1p-100f && fabsf(vdn) <= 0x1p40f) positive = ((f2u(vdm) ^ f2u(vdn)) >> 31) == 0u;
    else positive = (vdm / vdn) > 0.0f;
    if (!positive) return 0.0f;
    float r2 = roughness * roughness;
    float c2 = vdn * vdn;
    float t2 = fmaf(-vdn, vdn, 1.0f) / c2;  // (1 - c2) / c2, the product fused into the subtraction
    return 2.0f / (1.0f + sqrt_pt(fmaf(r2, t2, 1.0f)));
}

// Core/fresnel.h:11-49 (pow(x, 2.0f) -> x*x). tir_asin = asin(out_n / in_n), precomputed per material
// (DevMaterial::tir_front / tir_back; only read when in_n > out_n).
// refr_len2: DevConfig::refr_len2 (length(refr) <= 0.000005f as dot(refr, refr) <= refr_len2, exact).
__device__ __forceinline__ float fresnel_dielectric(v3 n, v3 in, float in_n, float out_n, v3 refr, float tir_asin,
                                                   float refr_len2) {
    float cos_in = dot(n, in * -1.0f);
    float cos_out = dot(-1.0f * n, refr);
    if (in_n > out_n && acos_pt(cos_in) >= tir_asin) return 1.0f;
    if (dot(refr, refr) <= refr_len2 || cos_out < 0) return 1.0f;
    float s = fmaf(in_n, cos_in, -(out_n * cos_out)) / fmaf(in_n, cos_in, out_n * cos_out);
    float p = fmaf(in_n, cos_out, -(out_n * cos_in)) / fmaf(in_n, cos_out, out_n * cos_in);
    return fmaf(s, s, p * p) / 2.0f;  // (s^2 + p^2) / 2
}

// Core/fresnel.h:51-76
__device__ __forceinline__ float fresnel_conductor(v3 n, v3 in, float eta, float k) {
    float cos_in = dot(n, in * -1.0f);
    float nk = fmaf(eta, eta, k * k);  // eta^2 + k^2
    float c2 = cos_in * cos_in;
    float two_n = 2 * eta;
    float two_n_c = two_n * cos_in;
    // (nk c2 - 2 eta c + 1) / (nk c2 + 2 eta c + 1): the left product of each sum fused
    float rs = (fmaf(nk, c2, -two_n_c) + 1.0f) / (fmaf(nk, c2, two_n_c) + 1.0f);
    // (nk - 2 eta c + c^2) / (nk + 2 eta c + c^2): each product fused in turn
    float rp = fmaf(cos_in, cos_in, fmaf(-two_n, cos_in, nk)) / fmaf(cos_in, cos_in, fmaf(two_n, cos_in, nk));
    return (rs + rp) / 2.0f;
}

// pixels[i] / 255.0f (texture.h:47-66), exactly: the product with RN(1/255), corrected by one FMA step
// with its exact residual. A plain multiply misses 126 of the 256 quotients; the corrected one
// reproduces all 256 (test_u8_quotients_are_exact checks every value on the device).
__device__ __forceinline__ float u8_unit(unsigned int b) {
    const float f = (float)b;
    const float c = 1.0f / 255.0f;
    const float q = f * c;
    const float r = fmaf(-q, 255.0f, f);
    return fmaf(r, c, q);
}

// A bilinear lookup issues its four texel loads at raised wave priority, as a walk step does its node loads
// (PT_WALK_PRIO below): round 5, C5 +0.2-0.35 %, C3 +0.25-0.37 %, metric +0.1-0.4 % (the sky's cube-map
// lookups), profiles/r05/prio/ab_tex.txt. Scheduling only.
#ifndef PT_TEX_PRIO
#define PT_TEX_PRIO 3
#endif

// One RGBA8 texel as a packed word; channels are converted one at a time where they are used, so a
// bilinear sample holds four words instead of twelve floats.
__device__ __forceinline__ unsigned int texel_raw(const uint8_t* px, int idx) {
    return *reinterpret_cast<const unsigned int*>(px + (size_t)idx * 4);
}
__device__ __forceinline__ float texel_c(unsigned int t, int c) { return u8_unit((t >> (8 * c)) & 0xffu); }
__device__ __forceinline__ float lerp1(float a, float b, float t) { return fmaf(t, b - a, a); }  // lerp, contracted

// Core/texture.h:15-79 (also the face lookup of Core/cube_map.h:20-119, same arithmetic)
__device__ __forceinline__ v3 sample_rgba8(const uint8_t* px, int w, int h, float au, float av, int bilinear) {
    if (bilinear) {
        float xr = au * (float)(w - 1);
        float yr = (1.0f - av) * (float)(h - 1);
        int fx = (int)clampf(floorf(xr), 0.0f, (float)(w - 1));
        int cx = (int)clampf(ceilf(xr), 0.0f, (float)(w - 1));
        int fy = (int)clampf(floorf(yr), 0.0f, (float)(h - 1));
        int cy = (int)clampf(ceilf(yr), 0.0f, (float)(h - 1));
        float lr = xr - floorf(xr);
        float bt = yr - floorf(yr);
#if PT_TEX_PRIO
        __builtin_amdgcn_s_setprio(PT_TEX_PRIO);  // until the four texel loads issue (PT_TEX_PRIO)
#endif
        const unsigned int t0 = texel_raw(px, fy * w + fx), t1 = texel_raw(px, fy * w + cx);
        const unsigned int t2 = texel_raw(px, cy * w + fx), t3 = texel_raw(px, cy * w + cx);
#if PT_TEX_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        float o[3];
#pragma unroll
        for (int c = 0; c < 3; c++)  // lerp(lerp(c0, c1, lr), lerp(c2, c3, lr), bt), one channel at a time
            o[c] = lerp1(lerp1(texel_c(t0, c), texel_c(t1, c), lr), lerp1(texel_c(t2, c), texel_c(t3, c), lr), bt);
        return mk3(o[0], o[1], o[2]);
    }
    int x = (int)clampf(au * (float)(w - 1), 0.0f, (float)(w - 1));
    int y = (int)clampf((1.0f - av) * (float)(h - 1), 0.0f, (float)(h - 1));
    const unsigned int t = texel_raw(px, y * w + x);
    return mk3(texel_c(t, 0), texel_c(t, 1), texel_c(t, 2));
}

// sample_rgba8 on texels already converted to floats (DevScene::cube_f): the same index arithmetic and
// lerps on the same values, without the per-sample byte conversions.
__device__ __forceinline__ v3 sample_f4(const float4* px, int w, int h, float au, float av, int bilinear) {
    if (bilinear) {
        float xr = au * (float)(w - 1);
        float yr = (1.0f - av) * (float)(h - 1);
        int fx = (int)clampf(floorf(xr), 0.0f, (float)(w - 1));
        int cx = (int)clampf(ceilf(xr), 0.0f, (float)(w - 1));
        int fy = (int)clampf(floorf(yr), 0.0f, (float)(h - 1));
        int cy = (int)clampf(ceilf(yr), 0.0f, (float)(h - 1));
        float lr = xr - floorf(xr);
        float bt = yr - floorf(yr);
#if PT_TEX_PRIO
        __builtin_amdgcn_s_setprio(PT_TEX_PRIO);  // until the four texel loads issue (PT_TEX_PRIO)
#endif
        const float4 t0 = px[fy * w + fx], t1 = px[fy * w + cx], t2 = px[cy * w + fx], t3 = px[cy * w + cx];
#if PT_TEX_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        return mk3(lerp1(lerp1(t0.x, t1.x, lr), lerp1(t2.x, t3.x, lr), bt),
                   lerp1(lerp1(t0.y, t1.y, lr), lerp1(t2.y, t3.y, lr), bt),
                   lerp1(lerp1(t0.z, t1.z, lr), lerp1(t2.z, t3.z, lr), bt));
    }
    int x = (int)clampf(au * (float)(w - 1), 0.0f, (float)(w - 1));
    int y = (int)clampf((1.0f - av) * (float)(h - 1), 0.0f, (float)(h - 1));
    const float4 t = px[y * w + x];
    return mk3(t.x, t.y, t.z);
}

__device__ __forceinline__ v3 sample_texture(const DevScene& sc, int id, v2 uv, int bilinear) {
    int4 d = sc.tex_desc[id];
    float au = uv.x - floorf(uv.x);
    float av = uv.y - floorf(uv.y);
    return sample_rgba8(sc.tex_pool + (size_t)(unsigned)d.z, d.x, d.y, au, av, bilinear);
}

// Core/cube_map.h:20-119
__device__ __forceinline__ v3 background(const DevScene& sc, const DevConfig& cfg, v3 d) {
    if (cfg.use_sky_box) {
        if (sc.cube_len <= 0) return mk3(0.0f, 0.0f, 0.0f);
        float u, v;
        int face;
        xyz_to_cube_uv(d.x, d.y, d.z, &face, &u, &v);
        int len = sc.cube_len;
        if (sc.cube_f) return sample_f4(sc.cube_f + (size_t)face * (size_t)len * (size_t)len, len, len, u, v, cfg.use_bilinear);
        const uint8_t* px = sc.cube + (size_t)face * (size_t)len * (size_t)len * 4;
        return sample_rgba8(px, len, len, u, v, cfg.use_bilinear);
    }
    if (cfg.use_sky) {
        float t = (dot(d, mk3(-0.41f, 0.41f, -0.82f)) + 1.0f) / 2.0f;
        v3 a = mk3(0.15f, 0.3f, 0.5f);
        v3 b = mk3(1.0f, 1.0f, 1.0f);
        return fma3(a, 1.0f - t, t * b) * 1.0f;  // ((1 - t) a + t b) * 1, the left product fused
    }
    return mk3(0.0f, 0.0f, 0.0f);
}

// Core/sphere.h:18-55 -> t only; the hit point/normal are derived for the winner afterwards.
__device__ __forceinline__ bool sphere_t(float4 s, v3 o, v3 d, float* t_out) {
    v3 op = mk3(s.x, s.y, s.z) - o;
    float b = dot(op, d);
    float delta = fmaf(s.w, s.w, fmaf(b, b, -dot(op, op)));  // (b b - op.op) + r r, contracted
    if (delta < 0) return false;
    float dr = sqrt_pt(delta);
    float t1 = b - dr;
    float t2 = b + dr;
    if (t1 < 0 && t2 < 0) return false;
    *t_out = (t1 > 0 && t2 > 0) ? fminf(t1, t2) : fmaxf(t1, t2);
    return true;
}

// Core/triangle.h:27-62 with edge1/edge2 precomputed (same IEEE subtraction, done once).
__device__ __forceinline__ bool triangle_test(float4 a, float4 b, float4 c, v3 o, v3 d, float* t, float* t1o, float* t2o) {
    v3 v0 = f4xyz(a), e1 = f4xyz(b), e2 = f4xyz(c);
    v3 p = cross(d, e2);
    float det = dot(e1, p);
    if (det == 0.0f) return false;
    float inv = rcp_exact(det);  // == 1.0f / det
    v3 tv = o - v0;
    v3 q = cross(tv, e1);
    float t1 = dot(tv, p) * inv;
    float t2 = dot(d, q) * inv;
    float tt = dot(e2, q) * inv;
    if (t1 >= 0.0f && t2 >= 0.0f && t1 + t2 <= 1.0f) {
        *t = tt; *t1o = t1; *t2o = t2;
        return true;
    }
    return false;
}

// Bvh/bounding_box.h:83-102 with 1/direction hoisted out of the node loop.
__device__ __forceinline__ bool box_hit(float4 lo, float4 hi, v3 o, v3 inv, float* entry) {
    float tx1 = (lo.x - o.x) * inv.x;
    float tx2 = (hi.x - o.x) * inv.x;
    float ty1 = (lo.y - o.y) * inv.y;
    float ty2 = (hi.y - o.y) * inv.y;
    float tz1 = (lo.z - o.z) * inv.z;
    float tz2 = (hi.z - o.z) * inv.z;
    float t_max = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    float t_min = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    *entry = t_max;
    return t_max <= t_min && t_min > 0.0f;
}

// Instrumentation (STATS kernels only): what one trace step touched, for the roofline model.
struct Counters {
    unsigned int nodes;       // BVH nodes fetched
    unsigned int tris;        // triangle tests
    unsigned int hit_mesh;    // closest hit on a triangle (shading reads normals/uvs/material)
    unsigned int hit_sphere;  // closest hit on a sphere
    unsigned int miss;        // escaped: background lookup
    unsigned int scatter;     // subsurface free-flight event (no surface shading)
};

// path_tracer_kernel.cu:85-161: stackless preorder walk with skip indices over one mesh, on the
// exact 32-B node records (the reference's own node sequence: the STATS kernels count its visits).
template <bool LEAF1, bool STATS>
__device__ __forceinline__ bool mesh_closest(const DevScene& sc, int begin, int end, v3 o, v3 d, v3 inv,
                                             float* ht, float* ht1, float* ht2, int* htri, Counters* ctr,
                                             float t0 = __builtin_inff()) {
    const __amdgpu_buffer_rsrc_t rn = make_rsrc(sc.nodes, sc.node_count * 32);
    const __amdgpu_buffer_rsrc_t rt = make_rsrc(sc.tri_geom, sc.tri_count * 48);
    float min_t = t0;  // infinity, or the medium bound (medium_bound)
    float min_t1 = 0.0f, min_t2 = 0.0f;
    int min_tri = -1;
    bool hit = false;
    int pos = begin;
    while (pos != end) {
        const float4 lo = bload(rn, pos * 32), hi = bload(rn, pos * 32 + 16);
        if (STATS) ctr->nodes++;
        float entry;
        if (box_hit(lo, hi, o, inv, &entry) && entry <= min_t) {
            const int slot = f2i(hi.w);
            if (slot >= 0) {
                if (LEAF1) {
                    float t, t1, t2;
                    if (STATS) ctr->tris++;
                    float4 a = bload(rt, slot * 48), b = bload(rt, slot * 48 + 16), c = bload(rt, slot * 48 + 32);
                    if (triangle_test(a, b, c, o, d, &t, &t1, &t2) && t > 0.0f && t < min_t) {
                        min_t = t; min_t1 = t1; min_t2 = t2; min_tri = slot; hit = true;
                    }
                } else {
                    for (int i = 0; i < sc.leaf_size; i++) {
                        int tri = sc.leaf_tris[slot + i];
                        if (tri == -1) break;
                        float t, t1, t2;
                        if (STATS) ctr->tris++;
                        float4 a = bload(rt, tri * 48), b = bload(rt, tri * 48 + 16), c = bload(rt, tri * 48 + 32);
                        if (triangle_test(a, b, c, o, d, &t, &t1, &t2) && t > 0.0f && t < min_t) {
                            min_t = t; min_t1 = t1; min_t2 = t2; min_tri = tri; hit = true;
                        }
                    }
                }
            }
            pos++;
        } else {
            pos = f2i(lo.w);
        }
    }
    if (hit) { *ht = min_t; *ht1 = min_t1; *ht2 = min_t2; *htri = min_tri; }
    return hit;
}

// The walk of mesh_closest one node at a time, for kernels that interleave walks with shading
// (pass_kernel_u): the state of one in-flight walk over one mesh, leaf size 1. Same node sequence,
// same tests, same acceptance rule as mesh_closest<true, false>.
struct MeshWalk {
    int pos, end;    // current node, end of the mesh's node range
    float t, t1, t2; // mesh-local closest hit (reference: the local min_t of intersect_triangle_mesh_bvh)
    int tri;         // -1 = no hit yet
};

// One step of the stackless preorder walk (path_tracer_kernel.cu:113-150) over a run of CHAIN
// consecutive records loaded together (the node and the next CHAIN - 1 in preorder). A passing internal
// node's successor is pos + 1 (its left child), whose record is then already in registers, so a descent
// costs no further dependent load. The visited nodes, their order and every test are the reference's;
// only more records are fetched per step (the extra ones beyond a failed test are not used). The walk
// stops at a leaf whose box passes (returns true with its triangle, not advanced): the lane's triangle
// test may then wait for a batch (pass_kernel_u), which changes nothing in its own sequence of tests.
template <int CHAIN>
struct ChainRecs {
    float4 lo[CHAIN], hi[CHAIN];
};
template <int CHAIN>
__device__ __forceinline__ void chain_load(const __amdgpu_buffer_rsrc_t rn, int pos, ChainRecs<CHAIN>& r) {
#pragma unroll
    for (int i = 0; i < CHAIN; i++) {
        r.lo[i] = bload(rn, (pos + i) * 32);
        r.hi[i] = bload(rn, (pos + i) * 32 + 16);
    }
    // Left alone, the compiler sinks the later records' loads into the branch that tests them, which
    // makes them a second dependent round trip. Using them here keeps all loads of the step issued
    // together (one round trip).
#pragma unroll
    for (int i = 1; i < CHAIN; i++) asm volatile("" ::"v"(r.lo[i].w), "v"(r.hi[i].w));
}
template <int CHAIN>
__device__ __forceinline__ bool chain_test(const ChainRecs<CHAIN>& r, v3 o, v3 inv, MeshWalk& w, int& tri) {
#pragma unroll
    for (int i = 0; i < CHAIN; i++) {
        float entry;
        if (box_hit(r.lo[i], r.hi[i], o, inv, &entry) && entry <= w.t) {
            const int slot = f2i(r.hi[i].w);
            if (slot >= 0) {
                tri = slot;
                return true;
            }
            w.pos++;
        } else {
            w.pos = f2i(r.lo[i].w);
            return false;
        }
    }
    return false;
}
template <int CHAIN>
__device__ __forceinline__ bool walk_box_chain(const __amdgpu_buffer_rsrc_t rn, v3 o, v3 inv, MeshWalk& w, int& tri) {
    ChainRecs<CHAIN> r;
    chain_load<CHAIN>(rn, w.pos, r);
    return chain_test<CHAIN>(r, o, inv, w, tri);
}

// Issue priority of a walk step from its start until its four loads are issued (s_setprio; pass_kernel_u raises
// it before walk_box_inline, which drops it to 0 right after the loads). Waves that stand ready to send a step's
// loads then win the SIMD's issue arbitration over waves in box tests, triangle batches or shading (31 % of wave
// cycles are issue stalls: SQ_WAIT_INST_ANY, profiles/r05/prio/), so the loads, the dependent chain that bounds
// the walk, start sooner. Scheduling only: the same instructions on the same values. Measured
// (profiles/r05/prio/ab.txt): metric 14547-14563 vs 14379-14384 Mrays/s, C4 +5.1 %, C5 +3.1 %, C3 +0.7 %; levels
// 1 and 2 gain about as much; priority held through the whole step loses (14282-14298), and so does a middle
// level (1 or 2) for the box tests after the loads issue (-1.3 %, profiles/r05/prio/ab_test_levels.txt).
#ifndef PT_WALK_PRIO
#define PT_WALK_PRIO 3
#endif

// The two-record step over the inline-leaf layout (pass_kernel_u, one triangle per leaf): a leaf is
// two records, its box record {lo, e2.z} {hi, slot} followed by its triangle {v0, e1.x} {e1.y, e1.z,
// e2.x, e2.y}; an internal record keeps {lo, skip} {hi, -1}. A leaf's skip is always the record after
// its triangle, so it needs no field. A step loads 64 B at pos as before: when pos is a leaf whose box
// passes, its triangle came with it (returned in a, e1, e2; the walk is not advanced). A leaf reached
// as the step's second record (the left child of a passing internal record) whose box passes ends the
// step without moving on: the next step tests it again (same inputs, same result) with its triangle.
// The nodes tested, their order and every test's outcome are the reference's.
__device__ __forceinline__ bool walk_box_inline(const __amdgpu_buffer_rsrc_t rn, v3 o, v3 inv, MeshWalk& w, int& tri,
                                                float4& a, float4& e1, float4& e2) {
    const float4 lo0 = bload(rn, w.pos * 32), hi0 = bload(rn, w.pos * 32 + 16);
    const float4 lo1 = bload(rn, w.pos * 32 + 32), hi1 = bload(rn, w.pos * 32 + 48);
#if PT_WALK_PRIO
    __builtin_amdgcn_s_setprio(0);  // the caller's raised issue priority ends once the step's loads are issued
#endif
    // one wait for all four loads (chain_load). Without it the compiler issues them in record order and tests
    // the first record after two (vmcnt(2)): the same registers and −0.2–0.6 % (profiles/r05/prio/ab_nopin.txt),
    // as the four 16-B pieces of one 64-B run return together
    asm volatile("" ::"v"(lo1.w), "v"(hi1.w));
    // the triangle operands of a first-record leaf, assigned on every step (they are read only after a
    // park): a conditional assignment makes the compiler merge old and new values through copies
    const int slot0 = f2i(hi0.w);
    tri = slot0;
    a = make_float4(lo1.x, lo1.y, lo1.z, 0.0f);
    e1 = make_float4(lo1.w, hi1.x, hi1.y, 0.0f);
    e2 = make_float4(hi1.z, hi1.w, lo0.w, 0.0f);
    // Both records' box tests always run and the next position is chosen by selects: the wave executed the
    // second record's test whenever any lane needed it anyway, and the nested branches cost exec-mask SALU
    // and branches on every step (31 % of wave cycles are issue stalls). Round 5: metric 14673-14700 vs
    // 14537-14567 Mrays/s, C4 +1.7 %, C5 +1.1 %, C3 +-0 (profiles/r05/select/ab.txt).
    float en0, en1;
    const bool p0 = box_hit(lo0, hi0, o, inv, &en0) && en0 <= w.t;
    const bool p1 = box_hit(lo1, hi1, o, inv, &en1) && en1 <= w.t;  // meaningful only when rec0 is internal
    const bool leaf0 = slot0 >= 0, leaf1 = f2i(hi1.w) >= 0;
    const int pos = w.pos;
    int skip0 = f2i(lo0.w), skip1 = f2i(lo1.w);
    asm("" : "+v"(skip0), "+v"(skip1));  // not loads, for the select-to-branch heuristic: the selects stay selects
    // rec0 fails: skip it (a leaf's skip is the record after its triangle). rec0 is a passing leaf: park (the
    // walk stays). rec0 is a passing internal record: rec1 is its left child; a passing leaf there ends the step
    // on it (tested again next step with its triangle), a passing internal rec1 descends, a failing one is skipped
    const int after1 = p1 ? (leaf1 ? pos + 1 : pos + 2) : (leaf1 ? pos + 3 : skip1);
    w.pos = p0 ? (leaf0 ? pos : after1) : (leaf0 ? pos + 2 : skip0);
    return p0 && leaf0;
}

// The leaf's triangle test (triangle.h:27-62, accepted when t > 0 && t < min_t, :128) with its records
// already loaded, then the walk moves past the leaf.
__device__ __forceinline__ void walk_tri_geom(float4 a, float4 b, float4 c, v3 o, v3 d, MeshWalk& w, int tri) {
    // triangle_test's arithmetic without its early return on det == 0 (1/det is then not used), the hit taken by
    // selects: the batch's instructions are the same, its exec-mask branches go (round 5: metric +0.6-1.0 %, C4
    // +0.8 %, C5 +0.5 %; profiles/r05/select/ab_tri_inside.txt). Running the test on every lane instead, with the
    // batch's own exec branch removed too, lost 1.5 % (ab_tri_merge.txt).
    v3 v0 = f4xyz(a), e1 = f4xyz(b), e2 = f4xyz(c);
    v3 p = cross(d, e2);
    float det = dot(e1, p);
    float inv = rcp_exact(det);  // == 1.0f / det
    v3 tv = o - v0;
    v3 q = cross(tv, e1);
    float t1 = dot(tv, p) * inv;
    float t2 = dot(d, q) * inv;
    float tt = dot(e2, q) * inv;
    const bool hit = det != 0.0f && t1 >= 0.0f && t2 >= 0.0f && t1 + t2 <= 1.0f && tt > 0.0f && tt < w.t;
    w.t = hit ? tt : w.t; w.t1 = hit ? t1 : w.t1; w.t2 = hit ? t2 : w.t2; w.tri = hit ? tri : w.tri;
    w.pos++;
}

// Per-path registers (the reference keeps these per pixel in HBM: rays, not_absorbed_colors,
// accumulated_colors, scatterings; path_tracer_kernel.cu:275-297). The scattering coefficients are
// always either the configuration's air values or some material's medium (they are only ever copied
// from out_medium, :594), so the path carries that material's id instead (-1 = air).
struct PathState {
    v3 o, d;
    v3 thr;
    v3 rad;
    int medium;
};

__device__ __forceinline__ void medium_coefficients(const DevScene& sc, const DevConfig& cfg, int medium, float sa[3],
                                                    float ss[3]) {
    if (medium < 0) {
        for (int c = 0; c < 3; c++) { sa[c] = cfg.air_absorption[c]; ss[c] = cfg.air_reduced_scattering[c]; }
    } else {
        const DevMaterial& M = sc.materials[medium];
        for (int c = 0; c < 3; c++) { sa[c] = M.absorption[c]; ss[c] = M.reduced_scattering[c]; }
    }
}

// init_data_kernel + generate_ray_kernel for one pixel (path_tracer_kernel.cu:275-379).
__device__ __forceinline__ void generate_path(const DevCamera& cam, const DevConfig& cfg, int pixel,
                                              int32_t hseed, PathState* ps) {
    ps->thr = mk3(1.0f, 1.0f, 1.0f);
    ps->rad = mk3(0.0f, 0.0f, 0.0f);
    ps->medium = -1;

    int image_y = (int)((float)pixel / cam.res_x);
    int image_x = (int)fmaf(-(float)image_y, cam.res_x, (float)pixel);  // pixel - image_y * res_x, contracted
    minstd rng = minstd_seed(mul_wrap(mul_wrap(hseed, hseed), hash_pt(pixel)));
    float jx = 0.0f, jy = 0.0f;
    if (cfg.use_anti_alias) {
        jx = minstd_uniform(&rng, -0.5f, 0.5f);
        jy = minstd_uniform(&rng, -0.5f, 0.5f);
    }
    v3 eye = mk3(cam.eye[0], cam.eye[1], cam.eye[2]);
    v3 view = mk3(cam.view[0], cam.view[1], cam.view[2]);
    v3 xa = mk3(cam.x_axis[0], cam.x_axis[1], cam.x_axis[2]);
    v3 ya = mk3(cam.y_axis[0], cam.y_axis[1], cam.y_axis[2]);
    float nx = fmaf(((float)image_x + jx) / (cam.res_x - 1.0f), 2.0f, -1.0f);
    float ny = fmaf(((float)image_y + jy) / (cam.res_y - 1.0f), 2.0f, -1.0f);
    v3 canvas = fma3(ya, ny, fma3(xa, nx, eye + view));      // ((eye + view) + nx xa) + ny ya
    v3 image_plane = fma3(normalize(canvas - eye), cam.focal, eye);  // eye + normalize(.) focal
    v3 ap;
    if (cam.aperture > 0.00001f) {
        float r1 = minstd_uniform(&rng, -0.5f, 0.5f) + 0.5f;
        float r2 = minstd_uniform(&rng, -0.5f, 0.5f) + 0.5f;
        float angle = r1 * kTWO_PI;
        float dist = cam.aperture * sqrt_pt(r2);
        float sa, ca;
        sincos_pt(angle, &sa, &ca);
        float ax = ca * dist;
        float ay = sa * dist;
        v3 hz = mk3(cam.horizontal[0], cam.horizontal[1], cam.horizontal[2]);
        v3 vt = mk3(cam.vertical[0], cam.vertical[1], cam.vertical[2]);
        ap = fma3(vt, ay, fma3(hz, ax, eye));  // (eye + ax hz) + ay vt
    } else {
        ap = eye;
    }
    ps->o = ap;
    ps->d = normalize(image_plane - ap);
}

// The kill test (path_tracer_kernel.cu:612-616, and :479-483 after a scatter): the reference ends a path
// iff length(thr) <= energy_exist_threshold, so a NaN throughput (NaN <= x is false) keeps the path going.
// Tested as !(dot(thr, thr) <= energy_len2), the same unordered outcome (DevConfig::energy_len2).
__device__ __forceinline__ bool alive_after(v3 thr, const DevConfig& cfg) {
    return !(dot(thr, thr) <= cfg.energy_len2);
}

// Closest hit over all spheres then every mesh BVH (path_tracer_kernel.cu:418-454).
struct Hit {
    float t, t1, t2;
    int type;  // 0 none, 1 sphere, 2 triangle
    int prim;
};

// t0: every mesh walk's starting min_t (infinity; the medium bound in the medium-bounded mode)
template <bool LEAF1, bool STATS>
__device__ __forceinline__ Hit closest_hit(const DevScene& sc, v3 o, v3 d, Counters* ctr, float t0 = __builtin_inff()) {
    Hit h;
    h.t = __builtin_inff(); h.t1 = __builtin_inff(); h.t2 = __builtin_inff();
    h.type = 0; h.prim = -1;
    for (int i = 0; i < sc.sphere_num; i++) {
        float t;
        if (sphere_t(sc.spheres[2 * i], o, d, &t) && t < h.t && t > 0.0f) {
            h.t = t; h.prim = i; h.type = 1;
        }
    }
    if (sc.mesh_num > 0) {
        v3 inv = mk3(rcp_exact(d.x), rcp_exact(d.y), rcp_exact(d.z));  // == 1.0f / d
        for (int m = 0; m < sc.mesh_num; m++) {
            const int2 r = uniform_ptr(sc.mesh_range)[m];
            float t, t1, t2;
            int tri;
            const bool mh = mesh_closest<LEAF1, STATS>(sc, r.x, r.y, o, d, inv, &t, &t1, &t2, &tri, ctr, t0);
            if (mh && t < h.t && t > 0.0f) {
                h.t = t; h.t1 = t1; h.t2 = t2; h.prim = tri; h.type = 2;
            }
        }
    }
    return h;
}

// The per-path part of the trace seed hash(seed) * hash(pixel) * hash(depth) (:415), int wrap.
__device__ __forceinline__ int32_t path_seed(int32_t hseed, int pixel) { return mul_wrap(hseed, hash_pt(pixel)); }

// The medium-bounded walk (pt_set_medium_bound / PT_MEDIUM_BOUND; a tolerance mode, off by default). A segment
// inside a scattering medium (:460-462) draws its free-flight distance first (:463-464) and scatters there
// when it is shorter than the closest hit (:466); intersection draws nothing, so the distance is known
// before the walk. A hit beyond it cannot matter, so each mesh walk may start with min_t = dist (1 + 2^-10)
// instead of infinity, which prunes every box entered beyond it. This equals the reference's walk whenever
// every box around an accepted triangle has a computed entry within that margin of the triangle's computed
// t; Moller-Trumbore on a ray grazing the triangle's plane has no such bound, so exactness is not proven.
// Measured: the whole C4 frame (72 M segments) renders bit-identical to the unbounded walk
// (profiles/r04/medium_bound/). Returns the walks' starting min_t: +inf outside a scattering medium.
__device__ __forceinline__ float medium_bound(const DevScene& sc, const DevConfig& cfg, int medium, int depth,
                                              int32_t pseed) {
    float sa[3], ss[3];
    medium_coefficients(sc, cfg, medium, sa, ss);
    if (ss[0] > 0.0f || dot(mk3(sa[0], sa[1], sa[2]), mk3(sa[0], sa[1], sa[2])) > cfg.sss_len2) {
        minstd rng = minstd_seed(mul_wrap(pseed, hash_pt(depth)));  // shade_hit's generator, first draw
        const float dist = -log_pt(minstd_uniform(&rng, 0.0f, 1.0f)) / ss[0];
        if (dist >= 0.0f && dist < __builtin_inff()) return dist + dist * 0x1p-10f;
    }
    return __builtin_inff();
}

// Scene features shade_hit can meet (pass_kernel_u is specialised on them: code a scene cannot reach is
// left out, which lowers the kernel's register peak). A feature left out must be unreachable for the
// scene: PT_FEAT_MEDIUM when no material (and not the configured air) has an absorption or reduced
// scattering coefficient other than 0 — the medium step is then never taken (:456-492); PT_FEAT_TEX when
// no material has a texture (:518-526).
#define PT_FEAT_MEDIUM 1
#define PT_FEAT_TEX 2
#define PT_FEAT_ALL 3
// PT_FEAT_MBOUND: the medium-bounded walk is on (pt_set_medium_bound; with PT_FEAT_MEDIUM only). Only these
// instances hold the walk's starting bound, one more register through the walk.
#define PT_FEAT_MBOUND 4

// The zero-specular shortcut's per-lane conditions (shade_hit): thr finite, |d|^2 and |n|^2 <= 1 + 2^-12, and
// the energy bound non-negative. Comparisons are false for NaN, so a NaN anywhere refuses the shortcut.
__device__ __forceinline__ bool spec_zero_ok(v3 thr, v3 d, v3 n, const DevConfig& cfg) {
    const float lim = 1.0f + 0x1p-12f;
    return dot(thr, thr) < __builtin_inff() && dot(d, d) <= lim && dot(n, n) <= lim && cfg.energy_len2 >= 0.0f;
}

template <bool STATS, int FEAT = PT_FEAT_ALL>
__device__ __forceinline__ bool shade_hit(const DevScene& sc, const DevConfig& cfg, int depth, int32_t pseed,
                                          PathState* ps, const Hit& h, Counters* ctr, unsigned long long* pc = nullptr);

// One invocation of trace_ray_kernel for one live ray (path_tracer_kernel.cu:381-625).
// pseed = path_seed(hash(pass), pixel). Returns false when the reference would write -1 into
// energy_exist_pixels.
// In the medium-bounded mode the walks start at the segment's medium bound, as in pass_kernel_u (so the
// instrumented kernel counts the bounded walk's nodes and triangle tests).
template <bool LEAF1, bool STATS>
__device__ __forceinline__ bool trace_step(const DevScene& sc, const DevConfig& cfg, int depth, int32_t pseed,
                                           PathState* ps, Counters* ctr) {
    const float t0 = cfg.medium_bound ? medium_bound(sc, cfg, ps->medium, depth, pseed) : __builtin_inff();
    const Hit h = closest_hit<LEAF1, STATS>(sc, ps->o, ps->d, ctr, t0);
    return shade_hit<STATS>(sc, cfg, depth, pseed, ps, h, ctr);
}

// The part of trace_ray_kernel after the closest hit is known (:456-624): medium, material,
// Fresnel-selected bounce, accumulation, kill test.
// pc (PT_UPROF builds): cycles spent per phase, added into pc[0..3] (medium, hit record or miss,
// Fresnel, bounce).
template <bool STATS, int FEAT>
__device__ __forceinline__ bool shade_hit(const DevScene& sc, const DevConfig& cfg, int depth, int32_t pseed,
                                          PathState* ps, const Hit& h, Counters* ctr, unsigned long long* pc) {
    unsigned long long tq = pc ? __builtin_readcyclecounter() : 0;
    auto mark = [&](int i) {
        if (pc) { const unsigned long long t = __builtin_readcyclecounter(); pc[i] += t - tq; tq = t; }
    };
    const float min_t = h.t;
    minstd rng = minstd_seed(mul_wrap(pseed, hash_pt(depth)));

    // medium: absorption and subsurface scattering (:456-492). A scattering lane replaces its ray in
    // place, and the rest of the step reads the ray back from *ps afterwards (below), so the
    // replaced and the original ray share registers instead of both living through the shading.
    if (FEAT & PT_FEAT_MEDIUM) {
        float sa[3], ss[3];
        medium_coefficients(sc, cfg, ps->medium, sa, ss);
        if (ss[0] > 0.0f || dot(mk3(sa[0], sa[1], sa[2]), mk3(sa[0], sa[1], sa[2])) > cfg.sss_len2) {
            float r = minstd_uniform(&rng, 0.0f, 1.0f);
            float dist = -log_pt(r) / ss[0];
            if (dist < min_t) {
                float r1 = minstd_uniform(&rng, 0.0f, 1.0f);
                float r2 = minstd_uniform(&rng, 0.0f, 1.0f);
                ps->o = fma3(ps->d, dist, ps->o);  // point_on_ray(dist) (ray.h:16), contracted
                ps->d = sample_sphere(r1, r2);
                ps->thr = ps->thr * absorption(sa, dist);
                if (STATS) ctr->scatter++;
                return alive_after(ps->thr, cfg);
            }
            ps->thr = ps->thr * absorption(sa, min_t);
        }
    }
    mark(0);
    const v3 o = ps->o, d = ps->d;

    if (STATS) { ctr->miss += h.type == 0; ctr->hit_sphere += h.type == 1; ctr->hit_mesh += h.type == 2; }
    if (h.type == 0) {  // miss (:618-624)
        v3 bg = background(sc, cfg, d);
        ps->rad = fma3v(ps->thr, bg, ps->rad);  // rad += thr * bg, contracted
        return false;
    }

    // material of the hit (:496-527); fields are read where they are used. The texture modulation
    // (:518-526) is applied in the branch that uses it (specular: reflect, diffuse: diffuse), from the
    // interpolated uv, so only uv stays live through Fresnel and the bounce choice.
    // the hit point, point_on_ray (ray.h:16; sphere.h:50 likewise), contracted. Without textures it is computed
    // where it is used (the sphere normal, the new origin) from o, d and min_t rather than held through the
    // Fresnel and bounce code: with the clamp bound computed at use (pt_kernels.hip) the bench kernel then fits
    // 64 VGPRs (8 waves) without spills. The textured kernel keeps it (C5 -0.5 % recomputed,
    // profiles/r04/knobs/waves_ab1.txt). The same value either way.
    constexpr bool lazy_point = !(FEAT & PT_FEAT_TEX);
    v3 held_point;
    if constexpr (!lazy_point) held_point = fma3(d, min_t, o);
    auto point = [&]() -> v3 {
        if constexpr (lazy_point) return fma3(d, min_t, o);
        else return held_point;
    };
    v3 normal;
    int mid;
    v2 uv = mk2(0.0f, 0.0f);
    bool textured = false;
    if (h.type == 1) {
        float4 s = sc.spheres[2 * h.prim];
        mid = f2i(sc.spheres[2 * h.prim + 1].x);
        normal = normalize(point() - mk3(s.x, s.y, s.z));
    } else {
        // the hit record's four 16-B loads through a buffer descriptor, issued together: the material id
        // (s3.w) arrives with the normals (a generic pointer here let the compiler merge it with the
        // sphere branch's LDS read into one flat load, a second round trip waiting on both counters)
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(sc.tri_shade, sc.tri_count * 64);
        const float4 s0 = bload(rs, h.prim * 64), s1 = bload(rs, h.prim * 64 + 16), s2 = bload(rs, h.prim * 64 + 32),
                     s3 = bload(rs, h.prim * 64 + 48);
        mid = f2i(s3.w);
        v3 n0 = mk3(s0.x, s0.y, s0.z), n1 = mk3(s0.w, s1.x, s1.y), n2 = mk3(s1.z, s1.w, s2.x);
        float w = 1.0f - h.t1 - h.t2;
        normal = fma3(n2, h.t2, fma3(n0, w, n1 * h.t1));  // (n0 w + n1 t1) + n2 t2, contracted
        const DevMaterial& M = sc.materials[mid];
        if ((FEAT & PT_FEAT_TEX) && (M.diffuse_texture_id != -1 || M.specular_texture_id != -1)) {
            v2 uv0 = mk2(s2.y, s2.z), uv1 = mk2(s2.w, s3.x), uv2 = mk2(s3.y, s3.z);
            uv = mk2(fmaf(uv2.x, h.t2, fmaf(uv0.x, w, uv1.x * h.t1)), fmaf(uv2.y, h.t2, fmaf(uv0.y, w, uv1.y * h.t1)));
            textured = true;
        }
    }
    const DevMaterial& M = sc.materials[mid];
    mark(1);
    // media on either side of the surface (:529-547)
    float in_n = cfg.air_n;
    float out_n = M.refraction_index;
    const bool transparent = M.is_transparent != 0;
    int out_medium = mid;
    if (dot(d, normal) > 0) {
        normal = normal * -1.0f;
        if (transparent) {
            float tn = in_n; in_n = out_n; out_n = tn;
            out_medium = -1;
        }
    }
    // in_n / out_n and out_n / in_n: the material's two ratios, swapped when the ray leaves it
    const float ratio_io = out_medium < 0 ? M.ratio_back : M.ratio_front;
    const float ratio_oi = out_medium < 0 ? M.ratio_front : M.ratio_back;
    v3 refr = refraction(normal, d, ratio_io);
    v3 bias_v = cfg.bias * normal;

    float R;
    const float k = M.extinction_coefficient;
    if (k == 0 || transparent) R = fresnel_dielectric(normal, d, in_n, out_n, refr, out_medium < 0 ? M.tir_back : M.tir_front, cfg.refr_len2);
    else R = fresnel_conductor(normal, d, out_n, k);

    mark(2);
    // Bounce (:563-610). The reflect and diffuse branches both draw r1, r2 right after r and build
    // their direction with the same hemisphere tail, so the draws and the tail are shared (a refract
    // lane draws them too and ignores them: the generator is local to this step).
    float r = minstd_uniform(&rng, 0.0f, 1.0f);
    const bool reflect = r < R;
    float r1 = minstd_uniform(&rng, 0.0f, 1.0f);
    float r2 = minstd_uniform(&rng, 0.0f, 1.0f);
    if (reflect || !transparent) {
        // A reflection off a material whose specular colour is (0, 0, 0) leaves thr * (spec * shadow) = thr * (+-0)
        // = +-0 whatever the sampled direction, provided thr and the shadow term are finite: the kill test
        // (:612-616) then ends the path with its radiance untouched (the reflect branch adds none), so the GGX
        // sample is not computed. Where thr * (0 * shadow) could be NaN the reference keeps the path, so the
        // shortcut needs (spec_zero_ok): thr finite; the shadow finite, which DevMaterial::spec_zero guarantees
        // with alpha in [2^-60, 4] as long as |d|^2 and |n|^2 are <= 1 + 2^-12 (then c2 = (v.n)^2 <= 1 + 2^-8,
        // so 1 + alpha^2 (1 - c2) / c2 >= 15/16 and the square root in ggx_g1 is finite; alpha^2 > 0 keeps
        // alpha^2 * inf = inf); and a non-negative energy bound, under which a zero throughput is killed.
        if (reflect && M.spec_zero && spec_zero_ok(ps->thr, d, normal, cfg)) return false;
        // both branches take sqrtf(r1) and one more square root: computed once for the batch, with the
        // second one's argument chosen per lane (a batch holds lanes of both kinds)
        const float s1 = sqrt_pt(r1);
        const float s2 = sqrt_pt(reflect ? 1.0f - r1 : fmaf(-s1, s1, 1.0f));
        float cos_t, sin_t;
        if (reflect) {  // sample_on_hemisphere_ggx_weight (:194-223), alpha = roughness^1.85 * 0.238 (:571)
            const float theta = atan_pt(M.rough_alpha * s1 / s2);  // alpha * sqrtf(r1) / sqrtf(1 - r1)
            sincos_pt(theta, &sin_t, &cos_t);
        } else {        // sample_on_hemisphere_cosine_weight (:163-192)
            cos_t = s1;  // sqrtf(r1)
            sin_t = s2;  // sqrtf(1 - cos_t * cos_t)
        }
        const v3 dir = hemisphere_dir(normal, cos_t, sin_t, r2);
        if (reflect) {  // reflection (:565-584)
            const float rough = M.rough_alpha;
            v3 mr = reflection(dir, d);
            float shadow = ggx_g1(rough, normal, dir, d) * ggx_g1(rough, normal, dir, mr);
            v3 spec = mk3(M.specular[0], M.specular[1], M.specular[2]);
            if (textured && M.specular_texture_id != -1)
                spec = spec * sample_texture(sc, M.specular_texture_id, uv, cfg.use_bilinear);
            ps->o = point() + bias_v;
            ps->d = mr;
            ps->thr = ps->thr * (spec * shadow);
        } else {        // diffuse (:597-610)
            v3 diff = mk3(M.diffuse[0], M.diffuse[1], M.diffuse[2]);
            if (textured && M.diffuse_texture_id != -1)
                diff = diff * sample_texture(sc, M.diffuse_texture_id, uv, cfg.use_bilinear);
            ps->rad = fma3v(ps->thr, mk3(M.emission[0], M.emission[1], M.emission[2]), ps->rad);  // +=, contracted
            ps->thr = ps->thr * diff;
            ps->o = point() + bias_v;
            ps->d = dir;
        }
    } else {  // refraction (:585-596)
        ps->o = point() - bias_v;
        ps->d = refr;
        ps->medium = out_medium;
        ps->thr = ps->thr * (ratio_oi * ratio_oi);  // ratio = out_n / in_n
    }
    mark(3);
    return alive_after(ps->thr, cfg);
}

// pixel_256_transform_gamma_corrected_kernel (path_tracer_kernel.cu:627-682) for one pixel.
__device__ __forceinline__ void store_u8(const DevConfig& cfg, v3 sum, int pass, uint8_t* out3) {
    v3 p = sum / (float)pass;
    float x, y, z;
    if (cfg.gamma_correction) {
        const float inv_gamma = 0.45454545f;
        x = clampf(exp_pt(inv_gamma * log_pt(p.x)) * 255.0f, 0.0f, 255.0f);
        y = clampf(exp_pt(inv_gamma * log_pt(p.y)) * 255.0f, 0.0f, 255.0f);
        z = clampf(exp_pt(inv_gamma * log_pt(p.z)) * 255.0f, 0.0f, 255.0f);
    } else {
        x = clampf(p.x * 255.0f, 0.0f, 255.0f);
        y = clampf(p.y * 255.0f, 0.0f, 255.0f);
        z = clampf(p.z * 255.0f, 0.0f, 255.0f);
    }
    out3[0] = (uint8_t)x;
    out3[1] = (uint8_t)y;
    out3[2] = (uint8_t)z;
}

}  // namespace pt
