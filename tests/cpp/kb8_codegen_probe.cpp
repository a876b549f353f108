// Codegen probe (test infrastructure): KannalaBrandt8::project(const Eigen::Vector3f&) and ::unproject(const
// cv::Point2f&) (src/CameraModels/KannalaBrandt8.cpp:67-84, 116-143) as plain scalar float code, built like the
// reference (g++ 11.4 -O3 with an FMA -march, CMakeLists.txt:10-13: GCC contracts a*b+c by default) and linked against
// this container's libm (glibc 2.35, the reference image's). tests/cpp/test_glibc_camera.cpp compares it with
// mam::cam::kb8_project_f / kb8_unproject_f, which place their fmas explicitly. The float parameters are read from a
// heap array, as mvParameters (std::vector<float>) is.
#include <math.h>

extern "C" void probe_kb8_project(const float* prm, float X, float Y, float Z, float* uo, float* vo) {
    const float rho2 = X * X + Y * Y;
    const float th = atan2f(sqrtf(rho2), Z);
    const float ang = atan2f(Y, X);
    const float th2 = th * th;
    const float th3 = th * th2;
    const float th5 = th3 * th2;
    const float th7 = th5 * th2;
    const float th9 = th7 * th2;
    const float rr = th + prm[4] * th3 + prm[5] * th5 + prm[6] * th7 + prm[7] * th9;
    *uo = prm[0] * rr * cosf(ang) + prm[2];
    *vo = prm[1] * rr * sinf(ang) + prm[3];
}

extern "C" void probe_kb8_unproject(const float* prm, float tol, float px, float py, float* out) {
    const float wx = (px - prm[2]) / prm[0], wy = (py - prm[3]) / prm[1];
    float sc = 1.f;
    float thd = sqrtf(wx * wx + wy * wy);
    thd = fminf(fmaxf(-3.1415926535897932384626433832795 / 2.f, thd), 3.1415926535897932384626433832795 / 2.f);
    if (thd > 1e-8) {
        float th = thd;
        for (int it = 0; it < 10; it++) {
            const float a2 = th * th, a4 = a2 * a2, a6 = a4 * a2, a8 = a4 * a4;
            const float e0 = prm[4] * a2, e1 = prm[5] * a4, e2 = prm[6] * a6, e3 = prm[7] * a8;
            const float step = (th * (1 + e0 + e1 + e2 + e3) - thd) / (1 + 3 * e0 + 5 * e1 + 7 * e2 + 9 * e3);
            th = th - step;
            if (fabsf(step) < tol) break;
        }
        sc = tanf(th) / thd;
    }
    out[0] = wx * sc;
    out[1] = wy * sc;
    out[2] = 1.f;
}
