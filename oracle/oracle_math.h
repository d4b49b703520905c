/*
 * oracle_math.h — TEST INFRASTRUCTURE (the parity checker), never shipped or measured.
 *
 * C restatement of the float helpers of the reference (Math/cuda_math.hpp) and of the
 * single-precision transcendentals that stand in for the CUDA intrinsics. Two math modes:
 *   OR_MATH_CEPHES (0): the Cephes single-precision algorithms with the fixed coefficients the
 *                       product documents; only IEEE +,-,*,/,sqrt, so with
 *                       -ffp-contract=off the result is bit-reproducible on any IEEE machine.
 *   OR_MATH_LIBM   (1): glibc sinf/cosf/tanf/atanf/asinf/acosf/expf/logf/powf (accurate libm),
 *                       i.e. what the reference CPU fallback calls (Core/path_tracer_cpu.cpp).
 * The image difference between the two modes calibrates how far a 1-ulp math change moves an
 * image, which is also the scale of the gap to the reference's __sinf/__powf hardware intrinsics.
 */
#ifndef ORACLE_MATH_H
#define ORACLE_MATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct { float x, y, z; } or_v3;

/* Contraction (DESIGN.md §5 "FMA contraction"). The reference's CUDA build contracts a*b+c into fused
 * multiply-adds (nvcc -fmad=true by default; gpu_path_tracer.vcxproj sets no --fmad=false): a product that is
 * an operand of an addition or subtraction in the same straight-line code is fused into it, the left product
 * where both operands are products, additions never reassociated. or_fma() writes out those sites; the rest
 * of this file is compiled with -ffp-contract=off. or_fma_on = 0 ("plain") evaluates the same sites unfused
 * (a*b rounded, then + c): the reference CPU fallback (MSVC /fp:precise on SSE2, no FMA) and an nvcc
 * --fmad=false build. Set once per render, before the parallel loops (oracle.c or_render_sig). */
static int or_fma_on = 1;
static inline float or_fma(float a, float b, float c) { return or_fma_on ? fmaf(a, b, c) : a * b + c; }

static inline or_v3 v3(float x, float y, float z) { or_v3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline or_v3 v_add(or_v3 a, or_v3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline or_v3 v_sub(or_v3 a, or_v3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline or_v3 v_mul(or_v3 a, or_v3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline or_v3 v_scale(or_v3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }   /* float3 * float */
static inline or_v3 s_scale(float s, or_v3 a) { return v3(s * a.x, s * a.y, s * a.z); }   /* float * float3 */
static inline or_v3 v_divs(or_v3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
/* a * s + c and a * b + c per component (the product fused into the addition that consumes it) */
static inline or_v3 v_fma(or_v3 a, float s, or_v3 c) { return v3(or_fma(a.x, s, c.x), or_fma(a.y, s, c.y), or_fma(a.z, s, c.z)); }
static inline or_v3 v_fmav(or_v3 a, or_v3 b, or_v3 c) { return v3(or_fma(a.x, b.x, c.x), or_fma(a.y, b.y, c.y), or_fma(a.z, b.z, c.z)); }
/* :1389 (a.x*b.x + a.y*b.y) + a.z*b.z, contracted */
static inline float v_dot(or_v3 a, or_v3 b) { return or_fma(a.z, b.z, or_fma(a.x, b.x, a.y * b.y)); }
static inline or_v3 v_cross(or_v3 a, or_v3 b) {                                                    /* :1581 */
    return v3(or_fma(a.y, b.z, -(a.z * b.y)), or_fma(a.z, b.x, -(a.x * b.z)), or_fma(a.x, b.y, -(a.y * b.x)));
}
static inline float v_len(or_v3 a) { return sqrtf(v_dot(a, a)); }                                   /* :1438 */
/* :1458 — host rsqrtf of cuda_math.hpp:33-36 is 1.0f / sqrtf(x); the device's rsqrtf under the CUDA
 * model (ck_rsqrt, defined below) */
static inline float ck_rsqrt(float x);
static __thread int or_ck_mode;
static inline or_v3 v_norm(or_v3 a) {
    float d = v_dot(a, a);
    float inv = or_ck_mode ? ck_rsqrt(d) : 1.0f / sqrtf(d);
    return v_scale(a, inv);
}
static inline or_v3 v_lerp(or_v3 a, or_v3 b, float t) { return v_fma(v_sub(b, a), t, a); }          /* :1260 */
static inline float or_clamp(float f, float a, float b) { return fmaxf(a, fminf(f, b)); }           /* :1290 */

static inline uint32_t or_f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float or_u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

#define OR_PI 3.1415926535897f
#define OR_TWO_PI 6.2831853071795f
#define OR_SQRT_ONE_THIRD 0.5773502691896f
#define OR_PIO2F 1.5707963267948966192f
#define OR_PIO4F 0.7853981633974483096f

/* ---- Cephes single precision (cephes/single: sinf.c, atanf.c, asinf.c, expf.c, logf.c) ---- */
static inline float c_ldexp(float x, int n) {
    if (n > 127) { x = x * or_u2f(0x7f000000u); n -= 127; }
    if (n < -126) { x = x * or_u2f(0x00800000u); n += 126; }
    if (n < -126) { x = x * or_u2f(0x00800000u); n += 126; }
    return x * or_u2f((uint32_t)(n + 127) << 23);
}

static inline float c_frexp(float x, int* e) {
    uint32_t u = or_f2u(x);
    int bias = 0;
    if ((u & 0x7f800000u) == 0) { x = x * 33554432.0f; u = or_f2u(x); bias = -25; }
    *e = (int)((u >> 23) & 0xffu) - 126 + bias;
    return or_u2f((u & 0x807fffffu) | 0x3f000000u);
}

static inline void c_sincos(float xx, float* so, float* co) {
    if (xx != xx) { *so = xx; *co = xx; return; }
    float x = xx;
    int ssign = 1, csign = 1;
    if (x < 0.0f) { x = -x; ssign = -1; }
    if (x > 8192.0f) x = 0.0f;
    int j = (int)(1.27323954473516f * x);        /* 4/pi */
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { ssign = -ssign; csign = -csign; j -= 4; }
    if (j > 1) csign = -csign;
    x = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    float z = x * x;
    float ps = ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x + x;
    float pc = ((2.443315711809948E-005f * z - 1.388731625493765E-003f) * z + 4.166664568298827E-002f) * z * z
               - 0.5f * z + 1.0f;
    float s = (j == 1 || j == 2) ? pc : ps;
    float c = (j == 1 || j == 2) ? ps : pc;
    *so = ssign < 0 ? -s : s;
    *co = csign < 0 ? -c : c;
}

static inline float c_atan(float xx) {
    float x = xx, y;
    int neg = x < 0.0f;
    if (neg) x = -x;
    if (x > 2.414213562373095f) { y = OR_PIO2F; x = -(1.0f / x); }
    else if (x > 0.4142135623730950f) { y = OR_PIO4F; x = (x - 1.0f) / (x + 1.0f); }
    else y = 0.0f;
    float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z - 3.33329491539E-1f) * z * x + x);
    return neg ? -y : y;
}

static inline float c_asin(float xx) {
    float a = xx < 0.0f ? -xx : xx;
    if (xx != xx) return xx;
    if (a > 1.0f) return or_u2f(0x7fc00000u);
    if (a < 1.0e-4f) return xx;
    float x, z;
    int flag = a > 0.5f;
    if (flag) { z = 0.5f * (1.0f - a); x = sqrtf(z); }
    else { x = a; z = x * x; }
    z = ((((4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z + 7.4953002686E-2f) * z
         + 1.6666752422E-1f) * z * x + x;
    if (flag) { z = z + z; z = OR_PIO2F - z; }
    return xx < 0.0f ? -z : z;
}

static inline float c_acos(float x) {
    if (x != x) return x;
    if (x < -1.0f || x > 1.0f) return or_u2f(0x7fc00000u);
    if (x < -0.5f) return 3.14159265358979f - 2.0f * c_asin(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * c_asin(sqrtf(0.5f * (1.0f - x)));
    return OR_PIO2F - c_asin(x);
}

static inline float c_exp(float x) {
    if (x != x) return x;
    if (x > 88.72283905206835f) return or_u2f(0x7f800000u);
    if (x < -103.278929903431851103f) return 0.0f;
    float z = floorf(1.44269504088896341f * x + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    int n = (int)z;
    z = x * x;
    z = (((((1.9875691500E-4f * x + 1.3981999507E-3f) * x + 8.3334519073E-3f) * x + 4.1665795894E-2f) * x
          + 1.6666665459E-1f) * x + 5.0000001201E-1f) * z + x + 1.0f;
    return c_ldexp(z, n);
}

static inline float c_log(float xx) {
    if (xx != xx) return xx;
    if (xx <= 0.0f) return xx == 0.0f ? or_u2f(0xff800000u) : or_u2f(0x7fc00000u);
    if (xx == or_u2f(0x7f800000u)) return xx;
    int e;
    float x = c_frexp(xx, &e);
    if (x < 0.707106781186547524f) { e -= 1; x = x + x - 1.0f; }
    else x = x - 1.0f;
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

/* ---- a model of the reference CUDA build's hardware intrinsics (tolerance calibration only) ----
 * OR_MATH_CUDA (2) / OR_MATH_CUDA_SITE (3). The reference calls __sinf, __cosf, __tanf, __expf, __logf
 * and __powf (path_tracer_kernel.cu:191,203-204,222,235,245-247,344-345,364-365,464,571,595,660-662) and
 * normalizes with rsqrtf (Math/cuda_math.hpp:1458-1462). Each is modelled as the exact value (double
 * libm) moved by the maximum error the CUDA C Programming Guide documents for it (intrinsic-function and
 * single-precision tables), in a direction drawn deterministically:
 *   __sinf / __cosf  absolute 2^-21.41 / 2^-21.19 on [-pi, pi], scaled by |x| / pi outside ("larger
 *                    otherwise": the hardware reduces the argument with a fixed-size 2pi)
 *   __expf           2 + floor(|1.173 x|) ulp
 *   __logf           absolute 2^-21.41 on [0.5, 2], else 3 ulp
 *   __powf(x, y)     exp2f(y * __log2f(x)) as the guide derives it: __log2f absolute 2^-22 on [0.5, 2],
 *                    else 2 ulp; the product rounded to float; the approximate exp2 2 ulp
 *   __tanf           __sinf(x) * (1 / __cosf(x)), as the guide derives it
 *   rsqrtf           2 ulp
 * atanf / asinf / acosf are the accurate CUDA functions there: glibc's (within 1 ulp) stands in.
 * OR_MATH_CUDA draws the direction from the function and the input bits (the hardware is a deterministic
 * function of its input: equal inputs in two pixels give equal outputs); OR_MATH_CUDA_SITE draws it from
 * (pass, pixel, depth, call number within the segment), the per-site model of verdict r02. */
#define OR_MATH_CEPHES 0
#define OR_MATH_LIBM 1
#define OR_MATH_CUDA 2
#define OR_MATH_CUDA_SITE 3

/* or_ck_mode (declared above v_norm): 0 off, else OR_MATH_CUDA / OR_MATH_CUDA_SITE for this thread */
static __thread uint64_t or_ck_key;       /* (pass, pixel, depth) of the segment being traced */
static __thread uint32_t or_ck_calls;     /* intrinsic calls so far in the segment */

static inline uint64_t or_ck_mix(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}
/* the segment key: set by the oracle before generate (depth -1) and before each trace step */
static inline void or_ck_segment(int mode, int pass, int pixel, int depth) {
    or_ck_mode = (mode == OR_MATH_CUDA || mode == OR_MATH_CUDA_SITE) ? mode : 0;
    or_ck_key = or_ck_mix(((uint64_t)(uint32_t)pass << 40) ^ ((uint64_t)(uint32_t)pixel << 8) ^ (uint64_t)(uint32_t)(depth + 1));
    or_ck_calls = 0;
}
/* +1 or -1 for a call of function `fn` on input bits `in` */
static inline int or_ck_sign(int fn, uint32_t in) {
    uint64_t h;
    if (or_ck_mode == OR_MATH_CUDA_SITE) h = or_ck_mix(or_ck_key ^ (0x9e3779b97f4a7c15ull * (uint64_t)(++or_ck_calls)));
    else h = or_ck_mix(((uint64_t)fn << 32) ^ (uint64_t)in ^ 0x632be59bd9b4e019ull);
    return (h >> 63) ? -1 : 1;
}
/* r moved by k ulps in direction s (finite non-zero r only) */
static inline float or_ck_ulps(float r, int k, int s) {
    if (!(r == r) || r == 0.0f || isinf(r)) return r;
    for (int i = 0; i < k; i++) r = nextafterf(r, s > 0 ? INFINITY : -INFINITY);
    return r;
}
static inline void ck_sincos(float x, float* so, float* co) {
    const double sc = fabs((double)x) > 3.14159265358979 ? fabs((double)x) / 3.14159265358979 : 1.0;
    *so = (float)(sin((double)x) + or_ck_sign(1, or_f2u(x)) * ldexp(1.0, -21) * pow(2.0, -0.41) * sc);
    *co = (float)(cos((double)x) + or_ck_sign(2, or_f2u(x)) * ldexp(1.0, -21) * pow(2.0, -0.19) * sc);
}
static inline float ck_exp(float x) {  /* __expf */
    return or_ck_ulps((float)exp((double)x), 2 + (int)floor(fabs(1.173 * (double)x)), or_ck_sign(3, or_f2u(x)));
}
static inline float ck_log(float x) {  /* __logf */
    if (!(x > 0.0f)) return logf(x);
    if (x >= 0.5f && x <= 2.0f) return (float)(log((double)x) + or_ck_sign(4, or_f2u(x)) * ldexp(1.0, -21) * pow(2.0, -0.41));
    return or_ck_ulps((float)log((double)x), 3, or_ck_sign(4, or_f2u(x)));
}
static inline float ck_log2(float x) {  /* __log2f */
    if (!(x > 0.0f)) return log2f(x);
    if (x >= 0.5f && x <= 2.0f) return (float)(log2((double)x) + or_ck_sign(5, or_f2u(x)) * ldexp(1.0, -22));
    return or_ck_ulps((float)log2((double)x), 2, or_ck_sign(5, or_f2u(x)));
}
static inline float ck_exp2(float y) {  /* ex2.approx */
    return or_ck_ulps((float)exp2((double)y), 2, or_ck_sign(6, or_f2u(y)));
}
static inline float ck_pow(float x, float y) {  /* __powf = exp2f(y * __log2f(x)) */
    if (x == 0.0f) return 0.0f;
    const float l = ck_log2(x);
    const float p = y * l;
    return ck_exp2(p);
}
static inline float ck_rsqrt(float x) {  /* rsqrtf */
    return or_ck_ulps((float)(1.0 / sqrt((double)x)), 2, or_ck_sign(7, or_f2u(x)));
}

/* ---- mode dispatch ---- */

#define OR_CK(mode) ((mode) == OR_MATH_CUDA || (mode) == OR_MATH_CUDA_SITE)
#define OR_ACCURATE(mode) ((mode) == OR_MATH_LIBM || OR_CK(mode))
static inline void m_sincos(int mode, float x, float* s, float* c) {
    if (mode == OR_MATH_LIBM) { *s = sinf(x); *c = cosf(x); }
    else if (OR_CK(mode)) ck_sincos(x, s, c);
    else c_sincos(x, s, c);
}
static inline float m_tan(int mode, float x) {
    if (mode == OR_MATH_LIBM) return tanf(x);
    float s, c;
    if (OR_CK(mode)) { ck_sincos(x, &s, &c); return s * (1.0f / c); }
    c_sincos(x, &s, &c);
    return s / c;
}
static inline float m_atan(int mode, float x) { return OR_ACCURATE(mode) ? atanf(x) : c_atan(x); }
static inline float m_asin(int mode, float x) { return OR_ACCURATE(mode) ? asinf(x) : c_asin(x); }
static inline float m_acos(int mode, float x) { return OR_ACCURATE(mode) ? acosf(x) : c_acos(x); }
static inline float m_exp(int mode, float x) { return mode == OR_MATH_LIBM ? expf(x) : (OR_CK(mode) ? ck_exp(x) : c_exp(x)); }
static inline float m_log(int mode, float x) { return mode == OR_MATH_LIBM ? logf(x) : (OR_CK(mode) ? ck_log(x) : c_log(x)); }
/* __powf(x, y) for x >= 0 */
static inline float m_pow(int mode, float x, float y) {
    if (mode == OR_MATH_LIBM) return powf(x, y);
    if (OR_CK(mode)) return ck_pow(x, y);
    if (x == 0.0f) return 0.0f;
    return c_exp(y * c_log(x));
}

#endif /* ORACLE_MATH_H */
