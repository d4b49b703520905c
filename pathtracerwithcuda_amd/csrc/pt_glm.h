// pt_glm.h — the glm 0.9.9 float matrix arithmetic the reference's host code uses on meshes
// (lib/glm: mat4 * vec4, mat4 * mat4, translate, scale, inverse, transpose), restated for both the
// host (scene builder, pt_host.cpp) and the device (the mesh refit kernel, pt_kernels.hip), so that a
// mesh transformed on either side rounds exactly as the reference's glm code does. Column-major like
// glm: c[col][row]; every expression keeps glm's evaluation order (contraction is off everywhere).
// Pinned against the real glm by tests/test_ref_pin.py (oracle/ref_harness.cpp).
#pragma once

#include <math.h>

#if defined(__HIPCC__)
#define PT_GLM_HD __host__ __device__ __forceinline__
#else
#define PT_GLM_HD inline
#endif

namespace ptglm {

struct M4 {
    float c[4][4];
};
struct V4 {
    float x, y, z, w;
};

PT_GLM_HD M4 identity4() {
    M4 m;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) m.c[i][j] = i == j ? 1.0f : 0.0f;
    return m;
}
PT_GLM_HD V4 add4(V4 a, V4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
PT_GLM_HD V4 mul4(V4 a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
PT_GLM_HD V4 mul4v(V4 a, V4 b) { return {a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }
PT_GLM_HD V4 sub4(V4 a, V4 b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
PT_GLM_HD V4 col(const M4& m, int i) { return {m.c[i][0], m.c[i][1], m.c[i][2], m.c[i][3]}; }
PT_GLM_HD void set_col(M4& m, int i, V4 v) { m.c[i][0] = v.x; m.c[i][1] = v.y; m.c[i][2] = v.z; m.c[i][3] = v.w; }

// operator*(mat4, vec4) (glm/detail/type_mat4x4.inl:487-524): (m0*x + m1*y) + (m2*z + m3*w)
PT_GLM_HD V4 mat_vec(const M4& m, V4 v) {
    return add4(add4(mul4(col(m, 0), v.x), mul4(col(m, 1), v.y)), add4(mul4(col(m, 2), v.z), mul4(col(m, 3), v.w)));
}

// operator*(mat4, mat4) (glm/detail/type_mat4x4.inl:581-599): column j = ((A0*b0 + A1*b1) + A2*b2) + A3*b3
PT_GLM_HD M4 mat_mul(const M4& a, const M4& b) {
    M4 r;
    for (int j = 0; j < 4; j++) {
        const V4 bj = col(b, j);
        set_col(r, j, add4(add4(add4(mul4(col(a, 0), bj.x), mul4(col(a, 1), bj.y)), mul4(col(a, 2), bj.z)),
                           mul4(col(a, 3), bj.w)));
    }
    return r;
}

// glm::translate(mat4(1), p) then glm::scale(., s) (glm/gtc/matrix_transform.inl:10-16, :50-59):
// the transform of Core/triangle_mesh.cpp:199-201 and :276-278
PT_GLM_HD M4 translate_scale(float px, float py, float pz, float sx, float sy, float sz) {
    M4 t = identity4();
    set_col(t, 3, add4(add4(add4(mul4(col(t, 0), px), mul4(col(t, 1), py)), mul4(col(t, 2), pz)), col(t, 3)));
    set_col(t, 0, mul4(col(t, 0), sx));
    set_col(t, 1, mul4(col(t, 1), sy));
    set_col(t, 2, mul4(col(t, 2), sz));
    return t;
}

// glm::inverse, generic 4x4 path (glm/detail/func_matrix.inl:296-355)
PT_GLM_HD M4 inverse4(const M4& M) {
    auto m = [&](int a, int b) { return M.c[a][b]; };
    float c00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3), c02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
    float c03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3);
    float c04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3), c06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3);
    float c07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
    float c08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2), c10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
    float c11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2);
    float c12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3), c14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3);
    float c15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
    float c16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2), c18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
    float c19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2);
    float c20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1), c22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1);
    float c23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
    V4 f0{c00, c00, c02, c03}, f1{c04, c04, c06, c07}, f2{c08, c08, c10, c11};
    V4 f3{c12, c12, c14, c15}, f4{c16, c16, c18, c19}, f5{c20, c20, c22, c23};
    V4 v0{m(1, 0), m(0, 0), m(0, 0), m(0, 0)}, v1{m(1, 1), m(0, 1), m(0, 1), m(0, 1)};
    V4 v2{m(1, 2), m(0, 2), m(0, 2), m(0, 2)}, v3{m(1, 3), m(0, 3), m(0, 3), m(0, 3)};
    V4 i0 = add4(sub4(mul4v(v1, f0), mul4v(v2, f1)), mul4v(v3, f2));
    V4 i1 = add4(sub4(mul4v(v0, f0), mul4v(v2, f3)), mul4v(v3, f4));
    V4 i2 = add4(sub4(mul4v(v0, f1), mul4v(v1, f3)), mul4v(v3, f5));
    V4 i3 = add4(sub4(mul4v(v0, f2), mul4v(v1, f4)), mul4v(v2, f5));
    const V4 sa{+1, -1, +1, -1}, sb{-1, +1, -1, +1};
    M4 inv;
    set_col(inv, 0, mul4v(i0, sa));
    set_col(inv, 1, mul4v(i1, sb));
    set_col(inv, 2, mul4v(i2, sa));
    set_col(inv, 3, mul4v(i3, sb));
    V4 row0{inv.c[0][0], inv.c[1][0], inv.c[2][0], inv.c[3][0]};
    V4 dot0 = mul4v(col(M, 0), row0);
    float dot1 = (dot0.x + dot0.y) + (dot0.z + dot0.w);
    float one_over_det = 1.0f / dot1;
    for (int i = 0; i < 4; i++) set_col(inv, i, mul4(col(inv, i), one_over_det));
    return inv;
}

PT_GLM_HD M4 transpose4(const M4& m) {
    M4 t;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) t.c[i][j] = m.c[j][i];
    return t;
}

// normalize with the host rsqrtf = 1 / sqrtf (Math/cuda_math.hpp:33-36, :1458-1462): the mesh code runs
// on the host in the reference
PT_GLM_HD void normalize3(float x, float y, float z, float* o) {
    const float inv = 1.0f / sqrtf(x * x + y * y + z * z);
    o[0] = x * inv;
    o[1] = y * inv;
    o[2] = z * inv;
}

}  // namespace ptglm
