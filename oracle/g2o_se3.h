// g2o_se3.h — TEST INFRASTRUCTURE ONLY (see orb_oracle.h header note).
//
// SE3Quat / Eigen quaternion arithmetic shared by the LocalBundleAdjustment and PoseOptimization oracles:
//   Thirdparty/g2o/g2o/types/se3quat.h  exp, operator*, map, normalizeRotation
//   Eigen QuaternionBase::_transformVector, quaternion_assign_impl<Matrix3>, toRotationMatrix
#pragma once

#include <cmath>

namespace oracle_g2o {

struct Quat { double x, y, z, w; };
struct SE3 { Quat r; double t[3]; };

inline void normalizeRotation(SE3& T) {
    if (T.r.w < 0) { T.r.x = -T.r.x; T.r.y = -T.r.y; T.r.z = -T.r.z; T.r.w = -T.r.w; }
    const double n = std::sqrt(T.r.x * T.r.x + T.r.y * T.r.y + T.r.z * T.r.z + T.r.w * T.r.w);
    T.r.x /= n; T.r.y /= n; T.r.z /= n; T.r.w /= n;
}

inline void cross(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// Eigen QuaternionBase::_transformVector
inline void quatRotate(const Quat& q, const double v[3], double o[3]) {
    const double qv[3] = {q.x, q.y, q.z};
    double uv[3];
    cross(qv, v, uv);
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    double c[3];
    cross(qv, uv, c);
    for (int i = 0; i < 3; i++) o[i] = v[i] + q.w * uv[i] + c[i];
}

inline Quat quatMul(const Quat& a, const Quat& b) {
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

inline void toRotationMatrix(const Quat& q, double R[9]) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

// Eigen quaternion_assign_impl<Matrix3>
inline Quat fromRotationMatrix(const double m[9]) {
    Quat q;
    const double t = m[0] + m[4] + m[8];
    if (t > 0) {
        double s = std::sqrt(t + 1.0);
        q.w = 0.5 * s;
        s = 0.5 / s;
        q.x = (m[7] - m[5]) * s;
        q.y = (m[2] - m[6]) * s;
        q.z = (m[3] - m[1]) * s;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = std::sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        double c[3];
        c[i] = 0.5 * s;
        s = 0.5 / s;
        q.w = (m[3 * k + j] - m[3 * j + k]) * s;
        c[j] = (m[3 * j + i] + m[3 * i + j]) * s;
        c[k] = (m[3 * k + i] + m[3 * i + k]) * s;
        q.x = c[0]; q.y = c[1]; q.z = c[2];
    }
    return q;
}

inline void mat3mul(const double A[9], const double B[9], double C[9]) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// SE3Quat::exp (se3quat.h)
inline SE3 se3Exp(const double u[6]) {
    const double omega[3] = {u[0], u[1], u[2]};
    const double upsilon[3] = {u[3], u[4], u[5]};
    const double theta = std::sqrt(omega[0] * omega[0] + omega[1] * omega[1] + omega[2] * omega[2]);
    const double Om[9] = {0, -omega[2], omega[1], omega[2], 0, -omega[0], -omega[1], omega[0], 0};
    double Om2[9];
    mat3mul(Om, Om, Om2);
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = ((i % 4 == 0) ? 1.0 : 0.0) + Om[i] + Om2[i];
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        const double a = std::sin(theta) / theta;
        const double b = (1 - std::cos(theta)) / (theta * theta);
        const double c = (theta - std::sin(theta)) / std::pow(theta, 3);
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4 == 0) ? 1.0 : 0.0;
            R[i] = I + a * Om[i] + b * Om2[i];
            V[i] = I + b * Om[i] + c * Om2[i];
        }
    }
    SE3 T;
    T.r = fromRotationMatrix(R);
    for (int i = 0; i < 3; i++) T.t[i] = V[3 * i] * upsilon[0] + V[3 * i + 1] * upsilon[1] + V[3 * i + 2] * upsilon[2];
    normalizeRotation(T);
    return T;
}

// SE3Quat::operator*
inline SE3 se3Mul(const SE3& a, const SE3& b) {
    SE3 r = a;
    double rt[3];
    quatRotate(a.r, b.t, rt);
    for (int i = 0; i < 3; i++) r.t[i] += rt[i];
    r.r = quatMul(a.r, b.r);
    normalizeRotation(r);
    return r;
}

inline void se3Map(const SE3& T, const double X[3], double o[3]) {
    quatRotate(T.r, X, o);
    for (int i = 0; i < 3; i++) o[i] += T.t[i];
}

}  // namespace oracle_g2o
