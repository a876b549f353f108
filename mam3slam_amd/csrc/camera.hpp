// camera.hpp — GeometricCamera models (include/mam_camera.h) evaluated identically on the host (oracle, C-ABI host
// code) and on gfx950. Built with -ffp-contract=off and correctly rounded f32 division / sqrt on both sides; every
// fused multiply-add below is an explicit fma, placed where the reference build's compiler puts one.
//
//   glibc_atanf / glibc_atan2f   glibc 2.35 sysdeps/ieee754/flt-32 s_atanf.c / e_atan2f.c (fdlibm; x86-64 has no FMA
//                                ifunc for them, so the generic SSE2 build). tests/cpp/test_glibc_camera.cpp checks
//                                them bit for bit against this container's libm (the reference image's glibc).
//   glibc_tanf                   glibc 2.35 tanf: the double-precision pi/2 reduction of sinf/cosf (reduce_fast) and
//                                fdlibm's __kernel_tanf; valid for |x| < 120 (unproject's theta is in [0, pi/2]).
//   kb8_project_f                KannalaBrandt8::project(const Eigen::Vector3f&) (KannalaBrandt8.cpp:67-84): the
//                                searches' projection. FMAs as g++ 11.4 -O3 -march=x86-64-v3 emits them (asm read:
//                                DESIGN.md §4): x*x + y*y -> fma(x, x, y*y), the odd polynomial as a chain of four
//                                fmas, fx*r*cos(psi) + cx -> fma(fx*r, cos, cx); cos/sin merged into sincosf.
//   kb8_unproject_f              KannalaBrandt8::unproject (KannalaBrandt8.cpp:116-143), same build: fma(pw.x, pw.x,
//                                pw.y^2), Newton numerator fma(theta, sum, -theta_d), denominator fma chain.
//   kb8_project_d / _jac_d       the Vector3d overloads (KannalaBrandt8.cpp:46-65, 145-175) of the g2o edges: float
//                                atan2f/sqrtf on the double point as the reference writes them, double polynomial and
//                                cos/sin (libm on the host, the device's double cos/sin on gfx950: within the 1e-4 BA
//                                budget, not bit-exact).
//   kb8_triangulate_matches_f    KannalaBrandt8::TriangulateMatches / Triangulate / epipolarConstrain
//                                (KannalaBrandt8.cpp:216-220, 306-406): Eigen 3.4 JacobiSVD<Matrix4f> (two-sided
//                                Jacobi sweeps, real_2x2_jacobi_svd, makeJacobi, descending sort, V.col(3)) restated
//                                without FMAs; 3-term Eigen reductions as e0 + (e1 + e2). The reference build's FMA
//                                placement inside Eigen's expression templates is not pinned (no Eigen here).
#pragma once

#include <stdint.h>

#include <cmath>

#include "../../include/mam_camera.h"
#include "det_math.hpp"

namespace mam {
namespace cam {

namespace detail {
MAM_HDI uint32_t fbits(float f) {
    union { float f; uint32_t u; } v;
    v.f = f;
    return v.u;
}
MAM_HDI float ffrom(uint32_t u) {
    union { float f; uint32_t u; } v;
    v.u = u;
    return v.f;
}
MAM_HDI float fabs_bits(float x) { return ffrom(fbits(x) & 0x7fffffffu); }
}  // namespace detail

// s_atanf.c
MAM_HDI float glibc_atanf(float x) {
    using namespace detail;
    const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f, atanhi2 = 9.8279368877e-01f,
                atanhi3 = 1.5707962513e+00f;
    const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f, atanlo2 = 3.4473217170e-08f,
                atanlo3 = 7.5497894159e-08f;
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const int32_t hx = (int32_t)fbits(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {   // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
    }
    if (ix < 0x3ee00000) {    // |x| < 0.4375
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = fabs_bits(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
    const float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
    z = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -z : z;
}

// e_atan2f.c
MAM_HDI float glibc_atan2f(float y, float x) {
    using namespace detail;
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)fbits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return glibc_atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            if (m == 0) return pi_o_4 + tiny;
            if (m == 1) return -pi_o_4 - tiny;
            if (m == 2) return 3.0f * pi_o_4 + tiny;
            return -3.0f * pi_o_4 - tiny;
        }
        if (m == 0) return 0.0f;
        if (m == 1) return -0.0f;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = glibc_atanf(fabs_bits(y / x));
    switch (m) {
        case 0: return z;
        case 1: return ffrom(fbits(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// k_tanf.c __kernel_tanf(x, y, iy), |x| <= pi/4 (+ the tail y)
MAM_HDI float glibc_kernel_tanf(float x, float y, int iy) {
    using namespace detail;
    const float T0 = 3.3333334327e-01f, T1 = 1.3333334029e-01f, T2 = 5.3968254477e-02f, T3 = 2.1869488060e-02f,
                T4 = 8.8632395491e-03f, T5 = 3.5920790397e-03f, T6 = 1.4562094584e-03f, T7 = 5.8804126456e-04f,
                T8 = 2.4646313977e-04f, T9 = 7.8179444245e-05f, T10 = 7.1407252108e-05f, T11 = -1.8558637748e-05f,
                T12 = 2.5907305826e-05f;
    const float pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
    const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    if (ix < 0x39000000) {   // |x| < 2^-13
        if ((int)x == 0) {
            if ((ix | (iy + 1)) == 0) return 1.0f / fabs_bits(x);
            if (iy == 1) return x;
            return -1.0f / (x + y);
        }
    }
    float z, r, v, w, s;
    if (ix >= 0x3f2ca140) {  // |x| >= 0.6744
        if (hx < 0) { x = -x; y = -y; }
        z = pio4 - x;
        w = pio4lo - y;
        x = z + w;
        y = 0.0f;
        if (fabs_bits(x) < 0x1p-13f) return (float)(1 - ((hx >> 30) & 2)) * (float)iy * (1.0f - 2 * iy * x);
    }
    z = x * x;
    w = z * z;
    r = T1 + w * (T3 + w * (T5 + w * (T7 + w * (T9 + w * T11))));
    v = z * (T2 + w * (T4 + w * (T6 + w * (T8 + w * (T10 + w * T12)))));
    s = z * x;
    r = y + z * (s * (r + v) + y);
    r += T0 * s;
    w = x + r;
    if (ix >= 0x3f2ca140) {
        v = (float)iy;
        return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
    }
    if (iy == 1) return w;
    // -1 / (x + r) computed with a split quotient
    z = ffrom(fbits(w) & 0xfffff000u);
    v = r - (z - x);
    const float a = -1.0f / w;
    const float t = ffrom(fbits(a) & 0xfffff000u);
    s = 1.0f + t * z;
    return t + a * (s + t * v);
}

MAM_HDI float glibc_tanf(float x) {
    using namespace detail;
    const int32_t ix = (int32_t)(fbits(x) & 0x7fffffffu);
    if (ix <= 0x3f490fda) return glibc_kernel_tanf(x, 0.0f, 1);
    // reduce_fast (sincosf.h, non-TOINT_INTRINSICS): n = nearest quadrant, r = x - n pi/2 in double
    const double xd = (double)x;
    const double rr = xd * glibc_detail::kHpiInv;
    const int n = ((int32_t)rr + 0x800000) >> 24;
    const double xr = xd - (double)n * glibc_detail::kHpi;
    const float y0 = (float)xr;
    const float y1 = (float)(xr - (double)y0);
    return glibc_kernel_tanf(y0, y1, 1 - ((n & 1) << 1));
}

// ------------------------------------------------------------------------------------------ projections (float)
MAM_HDI void pinhole_project_f(const mam_camera& c, float x, float y, float z, float* u, float* v) {
    *u = c.fx * x / z + c.cx;   // Pinhole::project(Vector3f) (Pinhole.cpp:35-41): no FMA site (division)
    *v = c.fy * y / z + c.cy;
}

MAM_HDI void kb8_project_f(const mam_camera& c, float x, float y, float z, float* u, float* v) {
    const float x2_plus_y2 = __builtin_fmaf(x, x, y * y);
    const float theta = glibc_atan2f(sqrtf(x2_plus_y2), z);
    const float psi = glibc_atan2f(y, x);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    float r = __builtin_fmaf(theta3, c.k[0], theta);
    r = __builtin_fmaf(theta5, c.k[1], r);
    r = __builtin_fmaf(theta7, c.k[2], r);
    r = __builtin_fmaf(theta9, c.k[3], r);
    float sp, cp;
    glibc_sincosf<true>(psi, &sp, &cp);
    *u = __builtin_fmaf(c.fx * r, cp, c.cx);
    *v = __builtin_fmaf(c.fy * r, sp, c.cy);
}

// GeometricCamera::project(const Eigen::Vector3f&)
MAM_HDI void project_f(const mam_camera& c, float x, float y, float z, float* u, float* v) {
    if (c.model == MAM_CAM_KANNALA_BRANDT8) kb8_project_f(c, x, y, z, u, v);
    else pinhole_project_f(c, x, y, z, u, v);
}

MAM_HDI void kb8_unproject_f(const mam_camera& c, float px, float py, float r[3]) {
    const float pwx = (px - c.cx) / c.fx, pwy = (py - c.cy) / c.fy;
    float scale = 1.0f;
    float theta_d = sqrtf(__builtin_fmaf(pwx, pwx, pwy * pwy));
    theta_d = fminf(fmaxf((float)(-3.1415926535897932384626433832795 / 2.f), theta_d),
                    (float)(3.1415926535897932384626433832795 / 2.f));
    if ((double)theta_d > 1e-8) {
        float theta = theta_d;
        for (int j = 0; j < 10; j++) {
            const float theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2,
                        theta8 = theta4 * theta4;
            const float k0t2 = c.k[0] * theta2, k1t4 = c.k[1] * theta4, k2t6 = c.k[2] * theta6,
                        k3t8 = c.k[3] * theta8;
            const float sum = (((1.0f + k0t2) + k1t4) + k2t6) + k3t8;
            const float num = __builtin_fmaf(theta, sum, -theta_d);
            const float den = __builtin_fmaf(
                k3t8, 9.0f, __builtin_fmaf(k2t6, 7.0f, __builtin_fmaf(k1t4, 5.0f, __builtin_fmaf(k0t2, 3.0f, 1.0f))));
            const float fix = num / den;
            theta = theta - fix;
            if (fabsf(fix) < c.precision) break;
        }
        scale = glibc_tanf(theta) / theta_d;
    }
    r[0] = pwx * scale;
    r[1] = pwy * scale;
    r[2] = 1.0f;
}

// ------------------------------------------------------------------------------------------ projections (double)
// GeometricCamera::project(const Eigen::Vector3d&) and projectJac (the g2o edges' error and Jacobian)
MAM_HDI void project_d(const mam_camera& c, const double X[3], double* u, double* v) {
    if (c.model != MAM_CAM_KANNALA_BRANDT8) {
        *u = (double)c.fx * X[0] / X[2] + (double)c.cx;
        *v = (double)c.fy * X[1] / X[2] + (double)c.cy;
        return;
    }
    const double x2_plus_y2 = X[0] * X[0] + X[1] * X[1];
    const double theta = (double)glibc_atan2f(sqrtf((float)x2_plus_y2), (float)X[2]);
    const double psi = (double)glibc_atan2f((float)X[1], (float)X[0]);
    const double theta2 = theta * theta;
    const double theta3 = theta * theta2;
    const double theta5 = theta3 * theta2;
    const double theta7 = theta5 * theta2;
    const double theta9 = theta7 * theta2;
    const double r = theta + (double)c.k[0] * theta3 + (double)c.k[1] * theta5 + (double)c.k[2] * theta7 +
                     (double)c.k[3] * theta9;
    *u = (double)c.fx * r * cos(psi) + (double)c.cx;
    *v = (double)c.fy * r * sin(psi) + (double)c.cy;
}

// J (row-major 2x3) = d project / d X
MAM_HDI void project_jac_d(const mam_camera& c, const double X[3], double J[6]) {
    if (c.model != MAM_CAM_KANNALA_BRANDT8) {
        // Pinhole::projectJac (Pinhole.cpp:71-81)
        J[0] = (double)c.fx / X[2];
        J[1] = 0.0;
        J[2] = -(double)c.fx * X[0] / (X[2] * X[2]);
        J[3] = 0.0;
        J[4] = (double)c.fy / X[2];
        J[5] = -(double)c.fy * X[1] / (X[2] * X[2]);
        return;
    }
    const double x2 = X[0] * X[0], y2 = X[1] * X[1], z2 = X[2] * X[2];
    const double r2 = x2 + y2;
    const double r = sqrt(r2);
    const double r3 = r2 * r;
    const double theta = atan2(r, X[2]);
    const double theta2 = theta * theta, theta3 = theta2 * theta;
    const double theta4 = theta2 * theta2, theta5 = theta4 * theta;
    const double theta6 = theta2 * theta4, theta7 = theta6 * theta;
    const double theta8 = theta4 * theta4, theta9 = theta8 * theta;
    const double k0 = c.k[0], k1 = c.k[1], k2 = c.k[2], k3 = c.k[3], fx = c.fx, fy = c.fy;
    const double f = theta + theta3 * k0 + theta5 * k1 + theta7 * k2 + theta9 * k3;
    const double fd = 1 + 3 * k0 * theta2 + 5 * k1 * theta4 + 7 * k2 * theta6 + 9 * k3 * theta8;
    J[0] = fx * (fd * X[2] * x2 / (r2 * (r2 + z2)) + f * y2 / r3);
    J[3] = fy * (fd * X[2] * X[1] * X[0] / (r2 * (r2 + z2)) - f * X[1] * X[0] / r3);
    J[1] = fx * (fd * X[2] * X[1] * X[0] / (r2 * (r2 + z2)) - f * X[1] * X[0] / r3);
    J[4] = fy * (fd * X[2] * y2 / (r2 * (r2 + z2)) + f * x2 / r3);
    J[2] = -fx * fd * X[0] / (r2 + z2);
    J[5] = -fy * fd * X[1] / (r2 + z2);
}

// ------------------------------------------------------------------------------------------ two-view triangulation
// Eigen JacobiRotation (Jacobi/Jacobi.h): (c, s); x' = c x + s y, y' = -s x + c y on a row / column pair
struct Rot {
    float c, s;
};

// JacobiRotation::makeJacobi(x, y, z) (real)
MAM_HDI Rot make_jacobi(float x, float y, float z) {
    const float fmin = 1.17549435e-38f;
    const float deno = 2.0f * fabsf(y);
    if (deno < fmin) return Rot{1.0f, 0.0f};
    const float tau = (x - z) / deno;
    const float w = sqrtf(tau * tau + 1.0f);
    const float t = tau > 0.0f ? 1.0f / (tau + w) : 1.0f / (tau - w);
    const float sign_t = t > 0.0f ? 1.0f : -1.0f;
    const float n = 1.0f / sqrtf(t * t + 1.0f);
    return Rot{n, -sign_t * (y / fabsf(y)) * fabsf(t) * n};
}

// JacobiSVD<Matrix4f> of A (row-major), the right singular vector of the smallest singular value (V.col(3) after
// the descending sort).
MAM_HDI void jacobi_svd4_v3(const float Ain[16], float vout[4]) {
    const float fmin = 1.17549435e-38f;          // considerAsZero
    const float precision = 2.0f * 1.1920929e-07f;  // 2 * NumTraits<float>::epsilon()
    float scale = 0.0f;
    for (int i = 0; i < 16; i++) scale = fmaxf(scale, fabsf(Ain[i]));
    if (scale == 0.0f) scale = 1.0f;
    float W[16], V[16];
    for (int i = 0; i < 16; i++) {
        W[i] = Ain[i] / scale;
        V[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    }
    float maxDiag = 0.0f;
    for (int i = 0; i < 4; i++) maxDiag = fmaxf(maxDiag, fabsf(W[5 * i]));
    bool finished = false;
    for (int sweep = 0; sweep < 64 && !finished; sweep++) {   // Eigen loops until converged; 64 sweeps never bind
        finished = true;
        for (int p = 1; p < 4; p++) {
            for (int q = 0; q < p; q++) {
                const float threshold = fmaxf(fmin, precision * maxDiag);
                if (fabsf(W[4 * p + q]) > threshold || fabsf(W[4 * q + p]) > threshold) {
                    finished = false;
                    // real_2x2_jacobi_svd (SVD/RealSvd2x2.h)
                    float m00 = W[4 * p + p], m01 = W[4 * p + q], m10 = W[4 * q + p], m11 = W[4 * q + q];
                    Rot rot1;
                    const float t = m00 + m11, d = m10 - m01;
                    if (fabsf(d) < fmin) {
                        rot1 = Rot{1.0f, 0.0f};
                    } else {
                        const float u = t / d;
                        const float tmp = sqrtf(1.0f + u * u);
                        rot1 = Rot{u / tmp, 1.0f / tmp};
                    }
                    {   // m.applyOnTheLeft(0, 1, rot1)
                        const float a0 = m00, a1 = m01, b0 = m10, b1 = m11;
                        m00 = rot1.c * a0 + rot1.s * b0;
                        m01 = rot1.c * a1 + rot1.s * b1;
                        m10 = -rot1.s * a0 + rot1.c * b0;
                        m11 = -rot1.s * a1 + rot1.c * b1;
                    }
                    const Rot jr = make_jacobi(m00, m01, m11);
                    // j_left = rot1 * j_right.transpose(); transpose = (c, -s); product (c1 c2 - s1 s2, c1 s2 + s1 c2)
                    const Rot jl{rot1.c * jr.c - rot1.s * (-jr.s), rot1.c * (-jr.s) + rot1.s * jr.c};
                    // W.applyOnTheLeft(p, q, j_left): rows p, q
                    if (!(jl.c == 1.0f && jl.s == 0.0f)) {
                        for (int k = 0; k < 4; k++) {
                            const float xi = W[4 * p + k], yi = W[4 * q + k];
                            W[4 * p + k] = jl.c * xi + jl.s * yi;
                            W[4 * q + k] = -jl.s * xi + jl.c * yi;
                        }
                    }
                    // W.applyOnTheRight(p, q, j_right) and V.applyOnTheRight(p, q, j_right): columns p, q with
                    // j_right.transpose() = (c, -s)
                    if (!(jr.c == 1.0f && jr.s == 0.0f)) {
                        const float c = jr.c, s = -jr.s;
                        for (int k = 0; k < 4; k++) {
                            const float xi = W[4 * k + p], yi = W[4 * k + q];
                            W[4 * k + p] = c * xi + s * yi;
                            W[4 * k + q] = -s * xi + c * yi;
                        }
                        for (int k = 0; k < 4; k++) {
                            const float xi = V[4 * k + p], yi = V[4 * k + q];
                            V[4 * k + p] = c * xi + s * yi;
                            V[4 * k + q] = -s * xi + c * yi;
                        }
                    }
                    maxDiag = fmaxf(maxDiag, fmaxf(fabsf(W[4 * p + p]), fabsf(W[4 * q + q])));
                }
            }
        }
    }
    // singular values |diag|, sorted descending with column swaps (first maximum: maxCoeff's first index)
    float sv[4];
    int col[4] = {0, 1, 2, 3};
    for (int i = 0; i < 4; i++) sv[i] = fabsf(W[5 * i]) * scale;
    for (int i = 0; i < 4; i++) {
        int pos = i;
        float mx = sv[i];
        for (int j = i + 1; j < 4; j++)
            if (sv[j] > mx) { mx = sv[j]; pos = j; }
        if (mx == 0.0f) break;
        if (pos != i) {
            const float ts = sv[i]; sv[i] = sv[pos]; sv[pos] = ts;
            const int tc = col[i]; col[i] = col[pos]; col[pos] = tc;
        }
    }
    for (int k = 0; k < 4; k++) vout[k] = V[4 * k + col[3]];
}

MAM_HDI float dot3(const float a[3], const float b[3]) { return a[0] * b[0] + (a[1] * b[1] + a[2] * b[2]); }

// KannalaBrandt8::TriangulateMatches (KannalaBrandt8.cpp:306-375): r1 / r2 = the unprojected rays of kp1 / kp2,
// R12 row-major, t12. Returns z1 (> 0) or -1..-5 as the reference does.
MAM_HDI float kb8_triangulate_matches(const mam_camera& c1, const mam_camera& c2, float kp1x, float kp1y,
                                      const float r1[3], float kp2x, float kp2y, const float r2[3], const float R12[9],
                                      const float t12[3], float sigmaLevel, float unc) {
    const float r21[3] = {R12[0] * r2[0] + (R12[1] * r2[1] + R12[2] * r2[2]),
                          R12[3] * r2[0] + (R12[4] * r2[1] + R12[5] * r2[2]),
                          R12[6] * r2[0] + (R12[7] * r2[1] + R12[8] * r2[2])};
    const float cosParallaxRays = dot3(r1, r21) / (sqrtf(dot3(r1, r1)) * sqrtf(dot3(r21, r21)));
    if ((double)cosParallaxRays > 0.9998) return -1.0f;
    // Tcw1 = [I | 0], Tcw2 = [R21 | -R21 t12], R21 = R12^T
    const float R21[9] = {R12[0], R12[3], R12[6], R12[1], R12[4], R12[7], R12[2], R12[5], R12[8]};
    float t2[3];
    for (int i = 0; i < 3; i++) t2[i] = (-R21[3 * i]) * t12[0] + ((-R21[3 * i + 1]) * t12[1] + (-R21[3 * i + 2]) * t12[2]);
    // Triangulate (KannalaBrandt8.cpp:394-406): A rows p.x T.row(2) - T.row(0), p.y T.row(2) - T.row(1)
    const float T1[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    const float T2[12] = {R21[0], R21[1], R21[2], t2[0], R21[3], R21[4], R21[5], t2[1], R21[6], R21[7], R21[8], t2[2]};
    float A[16];
    for (int j = 0; j < 4; j++) {
        A[j] = r1[0] * T1[8 + j] - T1[j];
        A[4 + j] = r1[1] * T1[8 + j] - T1[4 + j];
        A[8 + j] = r2[0] * T2[8 + j] - T2[j];
        A[12 + j] = r2[1] * T2[8 + j] - T2[4 + j];
    }
    float h[4];
    jacobi_svd4_v3(A, h);
    const float x3D[3] = {h[0] / h[3], h[1] / h[3], h[2] / h[3]};
    const float z1 = x3D[2];
    if (z1 <= 0.0f) return -2.0f;
    const float row2[3] = {R21[6], R21[7], R21[8]};
    const float z2 = dot3(row2, x3D) + t2[2];
    if (z2 <= 0.0f) return -3.0f;
    float u1, v1;
    kb8_project_f(c1, x3D[0], x3D[1], x3D[2], &u1, &v1);
    const float ex1 = u1 - kp1x, ey1 = v1 - kp1y;
    if ((double)(ex1 * ex1 + ey1 * ey1) > 5.991 * (double)sigmaLevel) return -4.0f;
    float X2[3];
    for (int i = 0; i < 3; i++) X2[i] = (R21[3 * i] * x3D[0] + (R21[3 * i + 1] * x3D[1] + R21[3 * i + 2] * x3D[2])) + t2[i];
    float u2, v2;
    kb8_project_f(c2, X2[0], X2[1], X2[2], &u2, &v2);
    const float ex2 = u2 - kp2x, ey2 = v2 - kp2y;
    if ((double)(ex2 * ex2 + ey2 * ey2) > 5.991 * (double)unc) return -5.0f;
    return z1;
}

// ------------------------------------------------------------------------------------------ SearchForTriangulation's
// per keyframe-pair geometry (ORBmatcher.cc:913-930): T12 = T1w * T2w^-1 (Sophus SE3f product, so3.hpp:325-340 +
// normalize :297-303, se3.hpp:208-211, 304-308), R12 = T12.rotationMatrix(), t12; the epipole ep = KF2's camera
// projection of KF1's centre C2 = T2w * Cw; for Pinhole pairs F12 = K1^T^-1 [t12]x R12 K2^-1 (Pinhole.cpp:107-112)
// with Eigen's 3x3 cofactor inverse. Poses are Sophus SE3f (unit quaternion x y z w, t).
MAM_HDI void quat_to_rot(const float q[4], float R[9]) {
    const float qx = q[0], qy = q[1], qz = q[2], qw = q[3];
    const float tx = 2.0f * qx, ty = 2.0f * qy, tz = 2.0f * qz;
    const float twx = tx * qw, twy = ty * qw, twz = tz * qw, txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    R[0] = 1.0f - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1.0f - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1.0f - (txx + tyy);
}

// SO3 action q * p (so3.hpp:358-367)
MAM_HDI void quat_act(const float q[4], const float p[3], float o[3]) {
    float u0 = q[1] * p[2] - q[2] * p[1], u1 = q[2] * p[0] - q[0] * p[2], u2 = q[0] * p[1] - q[1] * p[0];
    u0 += u0; u1 += u1; u2 += u2;
    const float c0 = q[1] * u2 - q[2] * u1, c1 = q[2] * u0 - q[0] * u2, c2 = q[0] * u1 - q[1] * u0;
    o[0] = (p[0] + q[3] * u0) + c0;
    o[1] = (p[1] + q[3] * u1) + c1;
    o[2] = (p[2] + q[3] * u2) + c2;
}

// Eigen compute_inverse<3x3> (LU/InverseImpl.h): cofactor(c, r) * (1 / det), row-major
MAM_HDI void inv3(const float m[9], float r[9]) {
#define MAM_COF(i, j) (m[3 * (((i) + 1) % 3) + ((j) + 1) % 3] * m[3 * (((i) + 2) % 3) + ((j) + 2) % 3] - \
                       m[3 * (((i) + 1) % 3) + ((j) + 2) % 3] * m[3 * (((i) + 2) % 3) + ((j) + 1) % 3])
    const float c0 = MAM_COF(0, 0), c1 = MAM_COF(1, 0), c2 = MAM_COF(2, 0);
    const float det = c0 * m[0] + (c1 * m[3] + c2 * m[6]);
    const float invdet = 1.0f / det;
    r[3] = MAM_COF(0, 1) * invdet;
    r[4] = MAM_COF(1, 1) * invdet;
    r[6] = MAM_COF(0, 2) * invdet;
    r[5] = MAM_COF(2, 1) * invdet;
    r[7] = MAM_COF(1, 2) * invdet;
    r[8] = MAM_COF(2, 2) * invdet;
    r[0] = c0 * invdet;
    r[1] = c1 * invdet;
    r[2] = c2 * invdet;
#undef MAM_COF
}

MAM_HDI void mul3(const float a[9], const float b[9], float o[9]) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) o[3 * i + j] = a[3 * i] * b[j] + (a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j]);
}

struct PairGeom {
    float R12[9], t12[3], F12[9], ep[2];
};

MAM_HDI void pair_geometry(const float q1[4], const float t1[3], const float q2[4], const float t2[3],
                           const mam_camera& c1, const mam_camera& c2, PairGeom* g) {
    // Tw2 = T2w^-1: conj(q2), conj(q2) * (-t2)
    const float qi2[4] = {-q2[0], -q2[1], -q2[2], q2[3]};
    const float mt2[3] = {t2[0] * -1.0f, t2[1] * -1.0f, t2[2] * -1.0f};
    float tw2[3];
    quat_act(qi2, mt2, tw2);
    // T12 = T1w * Tw2
    const float ax = q1[0], ay = q1[1], az = q1[2], aw = q1[3], bx = qi2[0], by = qi2[1], bz = qi2[2], bw = qi2[3];
    float q12[4] = {((aw * bx + ax * bw) + ay * bz) - az * by, ((aw * by + ay * bw) + az * bx) - ax * bz,
                    ((aw * bz + az * bw) + ax * by) - ay * bx, ((aw * bw - ax * bx) - ay * by) - az * bz};
    const float len = sqrtf((q12[0] * q12[0] + q12[1] * q12[1]) + (q12[2] * q12[2] + q12[3] * q12[3]));
    for (int k = 0; k < 4; k++) q12[k] = q12[k] / len;
    float a1[3];
    quat_act(q1, tw2, a1);
    for (int i = 0; i < 3; i++) g->t12[i] = t1[i] + a1[i];
    quat_to_rot(q12, g->R12);
    // Cw = T1w^-1 translation, C2 = T2w * Cw
    const float qi1[4] = {-q1[0], -q1[1], -q1[2], q1[3]};
    const float mt1[3] = {t1[0] * -1.0f, t1[1] * -1.0f, t1[2] * -1.0f};
    float Cw[3], C2[3];
    quat_act(qi1, mt1, Cw);
    quat_act(q2, Cw, C2);
    for (int i = 0; i < 3; i++) C2[i] = C2[i] + t2[i];
    project_f(c2, C2[0], C2[1], C2[2], &g->ep[0], &g->ep[1]);
    // F12 = ((K1^T^-1 [t12]x) R12) K2^-1
    const float tx[9] = {0.0f, -g->t12[2], g->t12[1], g->t12[2], 0.0f, -g->t12[0], -g->t12[1], g->t12[0], 0.0f};
    const float K1T[9] = {c1.fx, 0.0f, 0.0f, 0.0f, c1.fy, 0.0f, c1.cx, c1.cy, 1.0f};
    const float K2[9] = {c2.fx, 0.0f, c2.cx, 0.0f, c2.fy, c2.cy, 0.0f, 0.0f, 1.0f};
    float K1Ti[9], K2i[9], M1[9], M2[9];
    inv3(K1T, K1Ti);
    inv3(K2, K2i);
    mul3(K1Ti, tx, M1);
    mul3(M1, g->R12, M2);
    mul3(M2, K2i, g->F12);
}

}  // namespace cam
}  // namespace mam
