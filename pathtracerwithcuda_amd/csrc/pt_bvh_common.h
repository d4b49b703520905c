// pt_bvh_common.h — the Morton/Karras BVH arithmetic shared by the host builder (pt_host.cpp, g++)
// and the device builder (pt_bvh.hip, hipcc), so both produce the same tree bit for bit.
//
//   box of a triangle     Bvh/bounding_box.h:55-61 with cuda_math.hpp min/max(a, b, c) (:1180-1245)
//   box union             bounding_box::expand_to_fit_box (:34-39); the reference runs it on the host,
//                         where cuda_math.hpp's fminf/fmaxf are `a < b ? a : b` / `a > b ? a : b` (:13-21)
//   Morton code           Bvh/bvh.cpp:370-392 (bvh_morton_code_kernel.cu keeps the same arithmetic)
//   clz / split / range   Bvh/bvh.cpp:398-570, Kernel/bvh_morton_code_kernel.cu:14-254
#pragma once

#include <math.h>

#if defined(__HIPCC__)
#define PT_HD __host__ __device__
#else
#define PT_HD
#endif

namespace ptbvh {

struct Box {
    float lb[3], rt[3];
};

PT_HD inline Box box_of_vertices(const float* v0, const float* v1, const float* v2) {
    Box b;
    for (int k = 0; k < 3; k++) {
        float mn = v0[k], mx = v0[k];
        mn = v1[k] < mn ? v1[k] : mn;
        mn = v2[k] < mn ? v2[k] : mn;
        mx = v1[k] > mx ? v1[k] : mx;
        mx = v2[k] > mx ? v2[k] : mx;
        b.lb[k] = mn;
        b.rt[k] = mx;
    }
    return b;
}

PT_HD inline void expand(Box& a, const Box& b) {
    for (int k = 0; k < 3; k++) {
        a.lb[k] = a.lb[k] < b.lb[k] ? a.lb[k] : b.lb[k];
        a.rt[k] = a.rt[k] > b.rt[k] ? a.rt[k] : b.rt[k];
    }
}

// -0 -> +0 in every coordinate (x + 0.0f): PT_BVH_SAH's boxes, so that unions are the same in any order (the
// reference's a < b ? a : b keeps whichever of two zeros came last); no slab-test outcome depends on a zero's sign
PT_HD inline void canonical_zeros(Box& b) {
    for (int k = 0; k < 3; k++) {
        b.lb[k] = b.lb[k] + 0.0f;
        b.rt[k] = b.rt[k] + 0.0f;
    }
}

PT_HD inline bool is_thin(const Box& b) {  // bounding_box::is_thin_bounding_box
    return b.rt[0] == b.lb[0] || b.rt[1] == b.lb[1] || b.rt[2] == b.lb[2];
}

PT_HD inline unsigned int expand_bits(unsigned int v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

// fminf(fmaxf(p * 1024, 0), 1023); a NaN coordinate (zero mesh extent on an axis) maps to 0
PT_HD inline float clamp_1023(float v) {
    float x = v * 1024.0f;
    x = (x > 0.0f) ? x : 0.0f;  // NaN compares false -> 0
    return x < 1023.0f ? x : 1023.0f;
}

PT_HD inline unsigned int morton(float px, float py, float pz) {
    return expand_bits((unsigned int)clamp_1023(px)) * 4 + expand_bits((unsigned int)clamp_1023(py)) * 2 +
           expand_bits((unsigned int)clamp_1023(pz));
}

// (centroid - mesh.lb) / (mesh.rt - mesh.lb), centroid = 0.5 * (rt + lb)
PT_HD inline unsigned int morton_of_box(const Box& b, const Box& mesh) {
    float p[3];
    for (int k = 0; k < 3; k++) {
        const float c = 0.5f * (b.rt[k] + b.lb[k]);
        p[k] = (c - mesh.lb[k]) / (mesh.rt[k] - mesh.lb[k]);
    }
    return morton(p[0], p[1], p[2]);
}

PT_HD inline unsigned int clz32(unsigned int v) {  // Bvh/bvh.cpp:398-441 (table-driven; clz(0) = 32)
    return v == 0 ? 32u : (unsigned int)__builtin_clz(v);
}

// Bvh/bvh.cpp:446-481
template <class Codes>
PT_HD inline unsigned int find_split(const Codes& code, unsigned int first, unsigned int last) {
    const unsigned int fc = code[first], lc = code[last];
    if (fc == lc) return first;
    const unsigned int common = clz32(fc ^ lc);
    unsigned int split = first;
    unsigned int step = last - first;
    do {
        step = (step + 1) >> 1;
        const unsigned int ns = split + step;
        if (ns < last) {
            if (clz32(fc ^ code[ns]) > common) split = ns;
        }
    } while (step > 1);
    return split;
}

// Bvh/bvh.cpp:486-570, including its unsigned wrap-around and the equal-code run handling.
template <class Codes>
PT_HD inline void find_range(const Codes& code, unsigned int n, unsigned int index, unsigned int* rx, unsigned int* ry) {
    if (index == 0) { *rx = 0; *ry = n - 1; return; }
    const unsigned int initial = index;
    const unsigned int prev = code[index - 1], cur = code[index], next = code[index + 1];
    if (prev == cur && cur == next) {
        while (index > 0 && index < n - 1) {
            index++;
            if (index >= n - 1) break;
            if (code[index] != code[index + 1]) break;
        }
        *rx = initial; *ry = index;
        return;
    }
    int direction;
    unsigned int delta_min;
    const unsigned int left = clz32(cur ^ prev), right = clz32(cur ^ next);
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
        const int t = (int)(l_max / (unsigned int)divisor);
        test = index + (unsigned int)((l + t) * direction);
        if (test < n) {
            if (clz32(cur ^ code[test]) > delta_min) l = l + t;
        }
    }
    if (direction == 1) { *rx = index; *ry = index + (unsigned int)(l * direction); }
    else { *rx = index + (unsigned int)(l * direction); *ry = index; }
}

}  // namespace ptbvh
