// det_math.hpp — deterministic float/double scalar routines evaluated identically on host and gfx950
// (built with -ffp-contract=off, correctly rounded f32 division, no fast-math).
//
//   fast_atan2  : cv::fastAtan2 of OpenCV 4.5.4 (degrees), used by IC_Angle (reference
//                 src/ORBextractor.cc:102). Separate float ops, same order as the library.
//   det_sincos  : the (float)cos(angle) / (float)sin(angle) of computeOrbDescriptor
//                 (src/ORBextractor.cc:111-112). glibc's cosf/sinf cannot be replayed on the GPU, so the
//                 reference's value is replaced by a double-precision evaluation rounded once to float:
//                 Cody-Waite reduction by pi/2 and degree-15/16 Taylor polynomials, every step a separate
//                 IEEE double op. DESIGN.md §Parity policy records the residual difference to glibc.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define MAM_HDI __host__ __device__ __forceinline__
#else
#define MAM_HDI inline
#endif

namespace mam {

MAM_HDI float fast_atan2(float y, float x) {
    const float k = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k;
    const float p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k;
    const float p7 = -0.04432655554792128f * k;
    const float eps = (float)2.2204460492503131e-16;  // (float)DBL_EPSILON
    float ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

MAM_HDI void det_sincos(float af, float* s_out, float* c_out) {
    const double x = (double)af;
    const double TWO_OVER_PI = 0.63661977236758134308;
    const double P1 = 1.5707963267341256e+00;
    const double P2 = 6.0771005065061922e-11;
    const double P3 = 2.0222662487959506e-21;
    double t = x * TWO_OVER_PI;
#if defined(__HIP_DEVICE_COMPILE__)
    double n = __builtin_rint(t);
#else
    double n = __builtin_nearbyint(t);
#endif
    double r = x - n * P1;
    r = r - n * P2;
    r = r - n * P3;
    double r2 = r * r;
    double sp = -7.6471637318198164759e-13;
    sp = sp * r2 + 1.6059043836821614599e-10;
    sp = sp * r2 + -2.5052108385441718775e-08;
    sp = sp * r2 + 2.7557319223985890653e-06;
    sp = sp * r2 + -1.9841269841269841270e-04;
    sp = sp * r2 + 8.3333333333333333333e-03;
    sp = sp * r2 + -1.6666666666666666667e-01;
    double sr = r + (r * r2) * sp;
    double cp = 4.7794773323873852974e-14;
    cp = cp * r2 + -1.1470745597729724714e-11;
    cp = cp * r2 + 2.0876756987868098979e-09;
    cp = cp * r2 + -2.7557319223985890653e-07;
    cp = cp * r2 + 2.4801587301587301587e-05;
    cp = cp * r2 + -1.3888888888888888889e-03;
    cp = cp * r2 + 4.1666666666666666667e-02;
    cp = cp * r2 + -0.5;
    double cr = 1.0 + r2 * cp;
    long long q = (long long)n & 3;
    double s, c;
    if (q == 0) { s = sr; c = cr; }
    else if (q == 1) { s = cr; c = -sr; }
    else if (q == 2) { s = -sr; c = -cr; }
    else { s = -cr; c = sr; }
    *s_out = (float)s;
    *c_out = (float)c;
}

}  // namespace mam
