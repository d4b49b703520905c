// pt_math.h — vector algebra and single-precision transcendentals for the hot path.
//
// Reference: Math/cuda_math.hpp (float3 operators, dot :1389, length :1438, normalize :1458,
// cross :1581, lerp :1260, clamp :1300, convert_xyz_to_cube_uv :56-126) and the CUDA fast
// intrinsics the kernel calls (__sinf/__cosf/__tanf/__powf/__logf/__expf, accurate atanf /
// acosf / asinf; Kernel/path_tracer_kernel.cu:191,201-204,222,235,245-247,344-345,364-365,
// 464,571,595,660-662; Core/fresnel.h:28).
//
// Determinism contract: this file is compiled with -ffp-contract=off
// and without fast-math, so every +,-,*,/ and sqrtf is a single IEEE-754 correctly rounded
// operation on gfx950 exactly as on x86-64, and every fused multiply-add is written out as fmaf
// where the reference's CUDA build contracts one (nvcc's default -fmad=true; DESIGN.md §5 "FMA
// contraction"): a product that is an operand of an addition or subtraction in the same straight-
// line code is fused into it, the left product where both operands are products, and additions are
// never reassociated. The oracle writes the same fmaf at the same sites. The transcendentals below
// are Cephes single-precision algorithms with fixed coefficients, kept unfused (they stand in for
// the CUDA intrinsics, which are not source the compiler contracts), so a host restatement of the
// same algorithm reproduces the GPU bit-for-bit. normalize() uses 1/sqrtf (two correctly rounded
// ops) in place of the reference's rsqrtf approximation.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PT_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define PT_HD static inline
#endif

namespace pt {

struct v3 {
    float x, y, z;
};
struct v2 {
    float x, y;
};

PT_HD v3 mk3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
PT_HD v2 mk2(float x, float y) { v2 r; r.x = x; r.y = y; return r; }

PT_HD v3 operator+(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD v3 operator-(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD v3 operator*(v3 a, v3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_HD v3 operator*(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
PT_HD v3 operator*(float s, v3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
PT_HD v3 operator/(v3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
PT_HD v3 operator/(v3 a, v3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
PT_HD v3 operator/(float s, v3 a) { return mk3(s / a.x, s / a.y, s / a.z); }
PT_HD v2 operator+(v2 a, v2 b) { return mk2(a.x + b.x, a.y + b.y); }
PT_HD v2 operator*(v2 a, float s) { return mk2(a.x * s, a.y * s); }

// a * s + c per component (a float3 * float product fused into the addition that consumes it)
PT_HD v3 fma3(v3 a, float s, v3 c) { return mk3(fmaf(a.x, s, c.x), fmaf(a.y, s, c.y), fmaf(a.z, s, c.z)); }
// a * b + c per component
PT_HD v3 fma3v(v3 a, v3 b, v3 c) { return mk3(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z)); }

// cuda_math.hpp:1389, (a.x*b.x + a.y*b.y) + a.z*b.z contracted: the left product of the inner sum is fused
// with the right one, then the last product with the sum
PT_HD float dot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.x, b.x, a.y * b.y)); }
// cuda_math.hpp:1581, each a*b - c*d contracted as fmaf(a, b, -(c*d))
PT_HD v3 cross(v3 a, v3 b) {
    return mk3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
#if defined(__HIPCC__)
// 1.0f / x correctly rounded (the IEEE division of the reference and the oracle), from v_rcp_f32
// (1 ulp) refined by one Newton step with an exact FMA residual: 3 instructions instead of the 10 of
// the division sequence. test_rcp_exact_matches_division checks every significand in [1, 2) at several
// exponents; outside [2^-125, 2^125] (denormal or overflowing reciprocals, 0, inf, NaN) the division
// itself runs.
__device__ __forceinline__ float rcp_exact(float x) {
    const float ax = fabsf(x);
    if (ax >= 0x1p-125f && ax <= 0x1p125f) {
        const float r = __builtin_amdgcn_rcpf(x);
        const float e = fmaf(-x, r, 1.0f);
        return fmaf(e, r, r);
    }
    return 1.0f / x;
}
// sqrtf(x) correctly rounded, for x in [2^-96, inf): v_sqrt_f32 (within 1 ulp) then the two one-ulp
// residual checks of the compiler's own sqrtf expansion, without its scaling of small inputs and its
// class test for 0 / inf / NaN, which that range does not need. Elsewhere sqrtf itself runs.
// test_sqrt_exact_matches_sqrtf checks every significand at both exponent parities and the edges.
__device__ __forceinline__ float sqrt_exact(float x) {
    if (__float_as_uint(x) - 0x0f800000u < 0x70000000u) {  // 2^-96 <= x < inf
        const float s = __builtin_amdgcn_sqrtf(x);
        const float lo = __uint_as_float(__float_as_uint(s) - 1u), hi = __uint_as_float(__float_as_uint(s) + 1u);
        const float r = fmaf(-lo, s, x) <= 0.0f ? lo : s;
        return fmaf(-hi, s, x) > 0.0f ? hi : r;
    }
    return sqrtf(x);
}
#endif
// sqrtf: sqrt_exact on the device (the same correctly rounded value), the libm call on the host
PT_HD float sqrt_pt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return sqrt_exact(x);
#else
    return sqrtf(x);
#endif
}
// cuda_math.hpp:1438
PT_HD float length(v3 v) { return sqrt_pt(dot(v, v)); }
// cuda_math.hpp:1458 (rsqrtf -> 1/sqrtf, see header; on the device the reciprocal is rcp_exact, the
// same correctly rounded value)
PT_HD v3 normalize(v3 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    float inv_len = rcp_exact(sqrt_exact(dot(v, v)));
#else
    float inv_len = 1.0f / sqrtf(dot(v, v));
#endif
    return v * inv_len;
}
// cuda_math.hpp:1260, a + t*(b - a) contracted
PT_HD v3 lerp(v3 a, v3 b, float t) { return fma3(b - a, t, a); }
// cuda_math.hpp:1290,1300 (fmaxf(a, fminf(f, b)))
PT_HD float clampf(float f, float a, float b) { return fmaxf(a, fminf(f, b)); }
PT_HD v3 clamp3(v3 v, float a, float b) { return mk3(clampf(v.x, a, b), clampf(v.y, a, b), clampf(v.z, a, b)); }

// ---------------------------------------------------------------------------------------------
// bit helpers
PT_HD uint32_t f2u(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __float_as_uint(f);
#else
    uint32_t u; memcpy(&u, &f, 4); return u;
#endif
}
PT_HD float u2f(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __uint_as_float(u);
#else
    float f; memcpy(&f, &u, 4); return f;
#endif
}

constexpr float kPI = 3.1415926535897f;       // basic_math.hpp:14
constexpr float kTWO_PI = 6.2831853071795f;   // basic_math.hpp:16
constexpr float kE = 2.7182818284590f;        // basic_math.hpp:20
constexpr float kSQRT_ONE_THIRD = 0.5773502691896f;  // basic_math.hpp:21
constexpr float kPIO2F = 1.5707963267948966192f;
constexpr float kPIO4F = 0.7853981633974483096f;

// 2^n * x for n in [-276, 254]; exact-IEEE multiplies only.
PT_HD float ldexp_pt(float x, int n) {
    if (n > 127) { x = x * u2f(0x7f000000u); n -= 127; }   // 2^127
    if (n < -126) { x = x * u2f(0x00800000u); n += 126; }  // 2^-126
    if (n < -126) { x = x * u2f(0x00800000u); n += 126; }
    return x * u2f((uint32_t)(n + 127) << 23);
}

// x = m * 2^e with m in [0.5, 1); x finite and > 0
PT_HD float frexp_pt(float x, int* e) {
    uint32_t u = f2u(x);
    int bias = 0;
    if ((u & 0x7f800000u) == 0) {  // subnormal
        x = x * 33554432.0f;       // 2^25
        u = f2u(x);
        bias = -25;
    }
    *e = (int)((u >> 23) & 0xffu) - 126 + bias;
    return u2f((u & 0x807fffffu) | 0x3f000000u);
}

// Cephes sinf/cosf (single precision), combined reduction. Stands in for __sinf/__cosf.
PT_HD void sincos_pt(float xx, float* s_out, float* c_out) {
    const float FOPI = 1.27323954473516f;
    const float DP1 = 0.78515625f;
    const float DP2 = 2.4187564849853515625e-4f;
    const float DP3 = 3.77489497744594108e-8f;
    if (xx != xx) { *s_out = xx; *c_out = xx; return; }
    float x = xx;
    int sin_sign = 1;
    if (x < 0.0f) { x = -x; sin_sign = -1; }
    if (x > 8192.0f) { x = 0.0f; }  // out of the hot path's range; keeps the reduction exact
    int j = (int)(FOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    int cos_sign = 1;
    if (j > 3) { sin_sign = -sin_sign; cos_sign = -cos_sign; j -= 4; }
    if (j > 1) cos_sign = -cos_sign;
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    float sp = ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x + x;
    float cp = ((2.443315711809948E-005f * z - 1.388731625493765E-003f) * z + 4.166664568298827E-002f) * z * z
               - 0.5f * z + 1.0f;
    float s, c;
    if (j == 1 || j == 2) { s = cp; c = sp; } else { s = sp; c = cp; }
    *s_out = sin_sign < 0 ? -s : s;
    *c_out = cos_sign < 0 ? -c : c;
}

// Cephes atanf. Stands in for atanf (path_tracer_kernel.cu:201).
PT_HD float atan_pt(float xx) {
    float x = xx, y;
    int neg = 0;
    if (x < 0.0f) { neg = 1; x = -x; }
    if (x > 2.414213562373095f) { y = kPIO2F; x = -(1.0f / x); }
    else if (x > 0.4142135623730950f) { y = kPIO4F; x = (x - 1.0f) / (x + 1.0f); }
    else { y = 0.0f; }
    float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z - 3.33329491539E-1f) * z * x + x);
    return neg ? -y : y;
}

// Cephes asinf / acosf. Stand in for asinf/acosf (Core/fresnel.h:28).
PT_HD float asin_pt(float xx) {
    float a = xx < 0.0f ? -xx : xx;
    if (xx != xx) return xx;
    if (a > 1.0f) return u2f(0x7fc00000u);
    if (a < 1.0e-4f) return xx;
    float x, z;
    int flag;
    if (a > 0.5f) { z = 0.5f * (1.0f - a); x = sqrt_pt(z); flag = 1; }
    else { x = a; z = x * x; flag = 0; }
    z = ((((4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z + 7.4953002686E-2f) * z
         + 1.6666752422E-1f) * z * x + x;
    if (flag) { z = z + z; z = kPIO2F - z; }
    return xx < 0.0f ? -z : z;
}
PT_HD float acos_pt(float x) {
    if (x != x) return x;
    if (x < -1.0f || x > 1.0f) return u2f(0x7fc00000u);
    if (x < -0.5f) return 3.14159265358979f - 2.0f * asin_pt(sqrt_pt(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * asin_pt(sqrt_pt(0.5f * (1.0f - x)));
    return kPIO2F - asin_pt(x);
}

// Cephes expf. Stands in for __expf and __powf(E, .) (path_tracer_kernel.cu:245-247,660-662).
PT_HD float exp_pt(float x) {
    if (x != x) return x;
    if (x > 88.72283905206835f) return u2f(0x7f800000u);
    if (x < -103.278929903431851103f) return 0.0f;
    float z = floorf(1.44269504088896341f * x + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    int n = (int)z;
    z = x * x;
    z = (((((1.9875691500E-4f * x + 1.3981999507E-3f) * x + 8.3334519073E-3f) * x + 4.1665795894E-2f) * x
          + 1.6666665459E-1f) * x + 5.0000001201E-1f) * z + x + 1.0f;
    return ldexp_pt(z, n);
}

// Cephes logf. Stands in for __logf (path_tracer_kernel.cu:464,660-662).
PT_HD float log_pt(float xx) {
    if (xx != xx) return xx;
    if (xx <= 0.0f) return xx == 0.0f ? u2f(0xff800000u) : u2f(0x7fc00000u);
    if (xx == u2f(0x7f800000u)) return xx;
    int e;
    float x = frexp_pt(xx, &e);
    if (x < 0.707106781186547524f) { e -= 1; x = x + x - 1.0f; }
    else { x = x - 1.0f; }
    float z = x * x;
    float y = ((((((((7.0376836292E-2f * x - 1.1514610310E-1f) * x + 1.1676998740E-1f) * x - 1.2420140846E-1f) * x
                  + 1.4249322787E-1f) * x - 1.6668057665E-1f) * x + 2.0000714765E-1f) * x - 2.4999993993E-1f) * x
               + 3.3333331174E-1f) * x * z;
    float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    z = x + y;
    z = z + 0.693359375f * fe;
    return z;
}

// x^y for x >= 0 as exp(y log x). Stands in for __powf (path_tracer_kernel.cu:571).
PT_HD float pow_pt(float x, float y) {
    if (x == 0.0f) return 0.0f;
    return exp_pt(y * log_pt(x));
}

// tanf via the combined reduction. Stands in for __tanf (path_tracer_kernel.cu:344-345).
PT_HD float tan_pt(float x) {
    float s, c;
    sincos_pt(x, &s, &c);
    return s / c;
}

// cuda_math.hpp:56-126. index/maxAxis start defined so a NaN direction cannot index out of range.
PT_HD void xyz_to_cube_uv(float x, float y, float z, int* index, float* u, float* v) {
    float ax = fabsf(x), ay = fabsf(y), az = fabsf(z);
    int xp = x > 0 ? 1 : 0, yp = y > 0 ? 1 : 0, zp = z > 0 ? 1 : 0;
    float max_axis = 1.0f, uc = 0.0f, vc = 0.0f;
    int idx = 0;
    if (xp && ax >= ay && ax >= az) { max_axis = ax; uc = -z; vc = y; idx = 0; }
    if (!xp && ax >= ay && ax >= az) { max_axis = ax; uc = z; vc = y; idx = 1; }
    if (yp && ay >= ax && ay >= az) { max_axis = ay; uc = x; vc = -z; idx = 2; }
    if (!yp && ay >= ax && ay >= az) { max_axis = ay; uc = x; vc = z; idx = 3; }
    if (zp && az >= ax && az >= ay) { max_axis = az; uc = x; vc = y; idx = 4; }
    if (!zp && az >= ax && az >= ay) { max_axis = az; uc = -x; vc = y; idx = 5; }
    *u = 0.5f * (uc / max_axis + 1.0f);
    *v = 0.5f * (vc / max_axis + 1.0f);
    *index = idx;
}

// ---------------------------------------------------------------------------------------------
// RNG: path_tracer_kernel.cu:35-44 (hash, signed int with wrap-around and arithmetic >>) and
// thrust::default_random_engine = minstd_rand (a=48271, c=0, m=2^31-1) feeding
// uniform_real_distribution<float> (thrust/random/detail/uniform_real_distribution.inl:71-79).
PT_HD int32_t hash_pt(int32_t a_in) {
    uint32_t a = (uint32_t)a_in;
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (uint32_t)((int32_t)a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (uint32_t)((int32_t)a >> 16);
    return (int32_t)a;
}

// int32 product with two's-complement wrap (the reference relies on it; signed overflow is UB in C++)
PT_HD int32_t mul_wrap(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

struct minstd {
    uint32_t x;
};
// thrust linear_congruential_engine::seed (linear_congruential_engine.inl:42-50)
PT_HD minstd minstd_seed(int32_t s) {
    minstd r;
    uint32_t v = (uint32_t)s % 2147483647u;
    r.x = v == 0u ? 1u : v;
    return r;
}
PT_HD uint32_t minstd_next(minstd* e) {
    // x*48271 mod (2^31-1) by Mersenne folding: p < 2^47, (p & m) + (p >> 31) < 2^31 + 2^16,
    // so one conditional subtraction gives exactly p % m without a 64-bit division.
    const uint64_t p = (uint64_t)e->x * 48271ull;
    uint32_t r = (uint32_t)(p & 2147483647ull) + (uint32_t)(p >> 31);
    if (r >= 2147483647u) r -= 2147483647u;
    e->x = r;
    return e->x;
}
// uniform_real_distribution<float>(a, b): ((float)(x - min) / (1 + (float)(max - min))) * (b - a) + a
PT_HD float minstd_uniform(minstd* e, float a, float b) {
    float r = (float)(minstd_next(e) - 1u);
    r = r / (1.0f + 2147483645.0f);
    return r * (b - a) + a;
}

}  // namespace pt
