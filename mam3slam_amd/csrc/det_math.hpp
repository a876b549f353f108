// det_math.hpp — deterministic float/double scalar routines evaluated identically on host and gfx950
// (built with -ffp-contract=off, correctly rounded f32 division, no fast-math).
//
//   fast_atan2  : cv::fastAtan2 of OpenCV 4.5.4 (degrees), used by IC_Angle (reference
//                 src/ORBextractor.cc:102). Separate float ops, same order as the library.
//   glibc_sincosf<FMA> : the (float)cos(angle) / (float)sin(angle) of computeOrbDescriptor
//                 (src/ORBextractor.cc:111-112). With `using namespace std` both calls resolve to the float
//                 overloads, which g++ 11 -O3 merges into one sincosf call (asm checked: DESIGN.md §4); the
//                 reference image (ros:humble = Ubuntu 22.04, Dockerfile:18) links glibc 2.35, whose sincosf
//                 is sysdeps/ieee754/flt-32/sincosf.{c,h} + sincosf_data.c: reduce_fast by pi/2 in double
//                 (non-TOINT_INTRINSICS form: hpi_inv prescaled by 2^24, quadrant by integer truncation) and
//                 the degree-5/4 double polynomials of sincosf_poly. On x86-64 the ifunc picks the copy built
//                 with -mfma -mavx2 when the host has FMA + AVX2 (FMA = true: every a + b*c of the C source is
//                 one fused op, as GCC contracts it), else the SSE2 copy (FMA = false). Restated here op for op
//                 in IEEE double; host and gfx950 agree bit for bit (v_fma_f64 is the exact fused op).
//                 Valid for |y| < 120 (the reduce_fast range); rBRIEF angles are in [0, 2*pi].
//   det_sincos  : correctly rounded (float)cos/sin of the float argument evaluated in double (Cody-Waite
//                 reduction, Taylor polynomials). A non-default policy (MAM_FP_TRIG_CORRECTLY_ROUNDED).
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

namespace glibc_detail {
// sincosf_data.c __sincosf_table[0] (x86-64: TOINT_INTRINSICS = 0, so hpi_inv = 2/pi * 2^24)
constexpr double kHpiInv = 0x1.45F306DC9C883p+23;
constexpr double kHpi = 0x1.921FB54442D18p0;
constexpr double kC0 = 0x1p0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5,
                 kC3 = -0x1.6c087e89a359dp-10, kC4 = 0x1.99343027bf8c3p-16;
constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7, kS3 = -0x1.994eb3774cf24p-13;

// a*b + c as the FMA or SSE2 build of glibc evaluates it
template <bool FMA>
MAM_HDI double madd(double a, double b, double c) {
    if (FMA) return __builtin_fma(a, b, c);
    return a * b + c;   // two roundings (this file is compiled with -ffp-contract=off)
}

MAM_HDI uint32_t abstop12(float x) {
    union { float f; uint32_t u; } v;
    v.f = x;
    return (v.u >> 20) & 0x7ff;
}
}  // namespace glibc_detail

template <bool FMA>
MAM_HDI void glibc_sincosf(float y, float* sinp, float* cosp) {
    using namespace glibc_detail;
    double x = (double)y;
    int n = 0;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {          // |y| < pio4 by the top-12-bit test
        if (abstop12(y) < abstop12(0x1p-12f)) {
            *sinp = y;
            *cosp = 1.0f;
            return;
        }
    } else {
        // reduce_fast: r = x * hpi_inv; n = ((int32_t) r + 0x800000) >> 24; x - n * hpi
        const double r = x * kHpiInv;
        n = ((int32_t)r + 0x800000) >> 24;
        x = FMA ? __builtin_fma(-(double)n, kHpi, x) : x - (double)n * kHpi;
        if ((n & 3) == 1 || (n & 3) == 2) x = -x;           // sign[n & 3] = {1, -1, -1, 1}
    }
    // sincosf_poly(x * s, x * x, p, n): table 1 (n & 2) negates the cosine coefficients
    const double cs = (n & 2) ? -1.0 : 1.0;
    const double x2 = x * x;
    const double x4 = x2 * x2;
    const double x3 = x2 * x;
    const double c2 = madd<FMA>(x2, cs * kC4, cs * kC3);
    const double s1 = madd<FMA>(x2, kS3, kS2);
    const double c1 = madd<FMA>(x2, cs * kC1, cs * kC0);
    const double x5 = x3 * x2;
    const double x6 = x4 * x2;
    const double s = madd<FMA>(x3, kS1, x);
    const double c = madd<FMA>(x4, cs * kC2, c1);
    const float so = (float)madd<FMA>(x5, s1, s);
    const float co = (float)madd<FMA>(x6, c2, c);
    if (n & 1) {
        *sinp = co;
        *cosp = so;
    } else {
        *sinp = so;
        *cosp = co;
    }
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
