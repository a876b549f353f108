// se3.hpp — g2o SE3Quat / Eigen quaternion arithmetic on the device (FP64), as the reference evaluates it:
//   Thirdparty/g2o/g2o/types/se3quat.h   exp (Rodrigues R and V, small-angle branch), operator*, map,
//                                         normalizeRotation (w >= 0, unit)
//   Eigen QuaternionBase::_transformVector, quaternion_assign_impl<Matrix3> (Quaterniond(Matrix3d))
//   core/robust_kernel_impl.cpp:76-91    RobustKernelHuber::robustify
// Poses are 7 doubles: quaternion x, y, z, w then translation.
#pragma once

#include <hip/hip_runtime.h>

namespace mam {
namespace se3 {

__device__ __forceinline__ void quat_rotate(const double q[4], const double v[3], double o[3]) {
    double uv0 = q[1] * v[2] - q[2] * v[1], uv1 = q[2] * v[0] - q[0] * v[2], uv2 = q[0] * v[1] - q[1] * v[0];
    uv0 += uv0; uv1 += uv1; uv2 += uv2;
    const double c0 = q[1] * uv2 - q[2] * uv1, c1 = q[2] * uv0 - q[0] * uv2, c2 = q[0] * uv1 - q[1] * uv0;
    o[0] = v[0] + q[3] * uv0 + c0;
    o[1] = v[1] + q[3] * uv1 + c1;
    o[2] = v[2] + q[3] * uv2 + c2;
}

__device__ __forceinline__ void map_point(const double* T, const double* X, double o[3]) {
    quat_rotate(T, X, o);
    o[0] += T[4]; o[1] += T[5]; o[2] += T[6];
}

// RobustKernelHuber::robustify: rho[0], rho[1] (rho[2] is never read by the unary/binary edges)
__device__ __forceinline__ void huber(double e, double delta, double* r0, double* r1) {
    const double dsqr = delta * delta;
    if (e <= dsqr) { *r0 = e; *r1 = 1.0; }
    else {
        const double s = sqrt(e);
        *r0 = 2 * s * delta - dsqr;
        *r1 = delta / s;
    }
}

// Eigen Quaterniond(Matrix3d). The largest-diagonal branch is written out per case (static register indices: a
// runtime-indexed matrix would be placed in scratch memory).
template <int I>
__device__ __forceinline__ void rot_to_quat_case(const double m[9], double q[4]) {
    constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
    double s = sqrt(m[3 * I + I] - m[3 * J + J] - m[3 * K + K] + 1.0);
    q[I] = 0.5 * s;
    s = 0.5 / s;
    q[3] = (m[3 * K + J] - m[3 * J + K]) * s;
    q[J] = (m[3 * J + I] + m[3 * I + J]) * s;
    q[K] = (m[3 * K + I] + m[3 * I + K]) * s;
}

__device__ __forceinline__ void rot_to_quat(const double m[9], double q[4]) {
    const double t = m[0] + m[4] + m[8];
    if (t > 0) {
        double s = sqrt(t + 1.0);
        q[3] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (m[7] - m[5]) * s;
        q[1] = (m[2] - m[6]) * s;
        q[2] = (m[3] - m[1]) * s;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > (i == 1 ? m[4] : m[0])) i = 2;
        if (i == 0) rot_to_quat_case<0>(m, q);
        else if (i == 1) rot_to_quat_case<1>(m, q);
        else rot_to_quat_case<2>(m, q);
    }
}

__device__ __forceinline__ void normalize_q(double q[4]) {
    if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}

// O = exp(u) * T (VertexSE3Expmap::oplusImpl: SE3Quat::exp(update) * estimate())
__device__ __forceinline__ void exp_mul(const double u[6], const double T[7], double O[7]) {
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double Om[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double Om2[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) Om2[3 * r + c] = Om[3 * r] * Om[c] + Om[3 * r + 1] * Om[3 + c] + Om[3 * r + 2] * Om[6 + c];
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int k = 0; k < 9; k++) { R[k] = ((k % 4 == 0) ? 1.0 : 0.0) + Om[k] + Om2[k]; V[k] = R[k]; }
    } else {
        const double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
        const double c = (theta - sin(theta)) / (theta * theta * theta);
        for (int k = 0; k < 9; k++) {
            const double I = (k % 4 == 0) ? 1.0 : 0.0;
            R[k] = I + a * Om[k] + b * Om2[k];
            V[k] = I + b * Om[k] + c * Om2[k];
        }
    }
    double qe[4];
    rot_to_quat(R, qe);
    double te[3];
    for (int r = 0; r < 3; r++) te[r] = V[3 * r] * u[3] + V[3 * r + 1] * u[4] + V[3 * r + 2] * u[5];
    normalize_q(qe);
    double rt[3];
    quat_rotate(qe, T + 4, rt);
    double q[4];
    q[3] = qe[3] * T[3] - qe[0] * T[0] - qe[1] * T[1] - qe[2] * T[2];
    q[0] = qe[3] * T[0] + qe[0] * T[3] + qe[1] * T[2] - qe[2] * T[1];
    q[1] = qe[3] * T[1] + qe[1] * T[3] + qe[2] * T[0] - qe[0] * T[2];
    q[2] = qe[3] * T[2] + qe[2] * T[3] + qe[0] * T[1] - qe[1] * T[0];
    normalize_q(q);
    O[0] = q[0]; O[1] = q[1]; O[2] = q[2]; O[3] = q[3];
    O[4] = te[0] + rt[0]; O[5] = te[1] + rt[1]; O[6] = te[2] + rt[2];
}

}  // namespace se3
}  // namespace mam
