// rt_math.h -- float3 arithmetic with the exact operation order of glm 0.9.9.8 (non-SIMD build,
// the reference's pinned version: framework/cmake/download_framework_packages.cmake:19-22).
//
// Bit-parity with the reference needs:
//   * dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z          (glm compute_dot: tmp = a*b; x+y+z)
//   * cross    = (a.y*b.z - b.y*a.z, a.z*b.x - b.z*a.x, a.x*b.y - b.x*a.y)
//   * normalize(v) = v * (1.0f / sqrtf(dot(v,v)))       (glm inversesqrt = 1/sqrt)
//   * length(v) = sqrtf(dot(v,v)),  reflect(I,N) = I - (N*dot(N,I))*2
//   * glm::min(x,y) = (y < x) ? y : x, glm::max(x,y) = (x < y) ? y : x  (== std::min/max)
// Everything here is compiled with -ffp-contract=off, IEEE div/sqrt and denormals preserved
// (host g++ SSE2 scalar; device hipcc gfx950 defaults), so host and device produce identical
// bits for identical inputs.
#pragma once

#ifdef __HIPCC__
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

#include <math.h>

namespace rt {

struct v3 {
    float x, y, z;
};
struct v2 {
    float x, y;
};

RT_HD v3 mk(float x, float y, float z) { return v3{x, y, z}; }
RT_HD v3 splat(float s) { return v3{s, s, s}; }
RT_HD v3 operator+(v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_HD v3 operator-(v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_HD v3 operator*(v3 a, v3 b) { return v3{a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_HD v3 operator*(v3 a, float s) { return v3{a.x * s, a.y * s, a.z * s}; }
RT_HD v3 operator*(float s, v3 a) { return v3{s * a.x, s * a.y, s * a.z}; }
RT_HD v3 operator/(v3 a, float s) { return v3{a.x / s, a.y / s, a.z / s}; }
RT_HD v3 operator-(v3 a) { return v3{-a.x, -a.y, -a.z}; }
RT_HD v3& operator+=(v3& a, v3 b) {
    a = a + b;
    return a;
}

RT_HD float dot(v3 a, v3 b) {
    const float tx = a.x * b.x;
    const float ty = a.y * b.y;
    const float tz = a.z * b.z;
    return (tx + ty) + tz;
}
RT_HD v3 cross(v3 x, v3 y) {
    return v3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
RT_HD float length(v3 v) { return sqrtf(dot(v, v)); }
RT_HD v3 normalize(v3 v) { return v * (1.0f / sqrtf(dot(v, v))); }
RT_HD v3 reflect(v3 i, v3 n) { return i - (n * dot(n, i)) * 2.0f; }
RT_HD float gmin(float x, float y) { return (y < x) ? y : x; }
RT_HD float gmax(float x, float y) { return (x < y) ? y : x; }
RT_HD v3 gmin(v3 a, v3 b) { return v3{gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)}; }
RT_HD v3 gmax(v3 a, v3 b) { return v3{gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)}; }

// glm::quat * vec3 (glm/detail/type_quat.inl operator*(qua, vec3)).
RT_HD v3 quat_rotate(float qx, float qy, float qz, float qw, v3 v) {
    const v3 q = v3{qx, qy, qz};
    const v3 uv = cross(q, v);
    const v3 uuv = cross(q, uv);
    return v + ((uv * qw) + uuv) * 2.0f;
}

// glm::mat3 (column-major, m[col][row]) used by the spherical-light Rodrigues matrix.
struct m3 {
    float m[3][3];
};
// glm mat3 * vec3 (type_mat3x3.inl): row r = m[0][r]*v.x + m[1][r]*v.y + m[2][r]*v.z
RT_HD v3 mul(const m3& a, v3 v) {
    return v3{a.m[0][0] * v.x + a.m[1][0] * v.y + a.m[2][0] * v.z,
              a.m[0][1] * v.x + a.m[1][1] * v.y + a.m[2][1] * v.z,
              a.m[0][2] * v.x + a.m[1][2] * v.y + a.m[2][2] * v.z};
}
// glm mat3 * mat3: R[c][r] = A[0][r]*B[c][0] + A[1][r]*B[c][1] + A[2][r]*B[c][2]
RT_HD m3 mul(const m3& a, const m3& b) {
    m3 r;
    for (int c = 0; c < 3; ++c)
        for (int w = 0; w < 3; ++w)
            r.m[c][w] = a.m[0][w] * b.m[c][0] + a.m[1][w] * b.m[c][1] + a.m[2][w] * b.m[c][2];
    return r;
}

// shadow.cpp:134-137 rotatetionMatrix(angle, axis) with sinf/cosf of the (constant) angle
// supplied by the host: I + C*sin + (C*C)*(1-cos), each + element-wise left to right.
RT_HD m3 rodrigues(float sin_a, float one_minus_cos_a, v3 axis) {
    m3 c;
    c.m[0][0] = 0.0f;
    c.m[0][1] = axis.z;
    c.m[0][2] = -axis.y;
    c.m[1][0] = -axis.z;
    c.m[1][1] = 0.0f;
    c.m[1][2] = axis.x;
    c.m[2][0] = axis.y;
    c.m[2][1] = -axis.x;
    c.m[2][2] = 0.0f;
    const m3 cc = mul(c, c);
    m3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const float ident = (i == j) ? 1.0f : 0.0f;
            r.m[i][j] = (ident + c.m[i][j] * sin_a) + cc.m[i][j] * one_minus_cos_a;
        }
    return r;
}

}  // namespace rt
