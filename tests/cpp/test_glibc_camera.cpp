// Pins the camera restatements of mam3slam_amd/csrc/camera.hpp (shared by the oracle and gfx950) to this container's
// glibc 2.35 libm (the reference image's, ros:humble = Ubuntu 22.04) and to g++ 11.4's FMA contraction of the
// reference's KannalaBrandt8 code:
//   atanf  : every `stride`-th float of [0, +inf) and (-inf, 0]
//   atan2f : 4M random pairs (uniform, any-bit-pattern and tiny/huge ratios)
//   tanf   : every `stride`-th float of [-2.4, 2.4] (unproject's theta range is [0, pi/2])
//   kb8_project_f / kb8_unproject_f : against kb8_codegen_probe.cpp built with -O3 -march=x86-64-v3, over random
//            points in front of the test-YAML camera (test/settingsForTest_00.yaml) and random pixels of its image.
// Prints "OK ..." and exits 0 when everything is bit-exact.
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>

#include "../../mam3slam_amd/csrc/camera.hpp"

extern "C" void probe_kb8_project(const float* prm, float X, float Y, float Z, float* uo, float* vo);
extern "C" void probe_kb8_unproject(const float* prm, float tol, float px, float py, float* out);

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float from(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv) {
    const uint32_t stride = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 10) : 1;
    void* m = dlopen("libm.so.6", RTLD_NOW);
    auto latanf = (float (*)(float))dlsym(m, "atanf");
    auto latan2f = (float (*)(float, float))dlsym(m, "atan2f");
    auto ltanf = (float (*)(float))dlsym(m, "tanf");
    if (!latanf || !latan2f || !ltanf) { printf("FAIL dlsym\n"); return 2; }
    unsigned long long bad_atan = 0, bad_atan2 = 0, bad_tan = 0, bad_proj = 0, bad_unproj = 0, n = 0;
    for (uint64_t u = 0; u < 0x7f800000ull; u += stride) {
        for (uint32_t s = 0; s < 2; s++) {
            const float x = from((uint32_t)u | (s << 31));
            if (bits(latanf(x)) != bits(mam::cam::glibc_atanf(x))) bad_atan++;
            n++;
        }
    }
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(-2000.f, 2000.f);
    for (int i = 0; i < 4000000; i++) {
        float y, x;
        if (i % 3 == 0) { y = U(rng); x = U(rng); }
        else if (i % 3 == 1) { y = from(rng()); x = from(rng()); if (y != y || x != x) continue; }
        else { y = U(rng) * 1e-3f; x = U(rng); }
        if (bits(latan2f(y, x)) != bits(mam::cam::glibc_atan2f(y, x))) bad_atan2++;
    }
    const uint32_t hi = bits(2.4f);
    for (uint32_t u = 0; u <= hi; u += stride) {
        const float x = from(u);
        if (bits(ltanf(x)) != bits(mam::cam::glibc_tanf(x))) bad_tan++;
        if (bits(ltanf(-x)) != bits(mam::cam::glibc_tanf(-x))) bad_tan++;
    }
    // test/settingsForTest_00.yaml: KannalaBrandt8, 960 x 960
    float* prm = (float*)malloc(8 * sizeof(float));
    const float init[8] = {322.7022465231787f, 322.25818444649866f, 473.48961846063645f, 484.62594873664256f,
                           0.052348933344686564f, 0.014590092715993354f, -0.030877354788616376f, 0.00650873486325155f};
    memcpy(prm, init, sizeof(init));
    mam_camera cam{};
    cam.fx = prm[0]; cam.fy = prm[1]; cam.cx = prm[2]; cam.cy = prm[3];
    for (int k = 0; k < 4; k++) cam.k[k] = prm[4 + k];
    cam.model = MAM_CAM_KANNALA_BRANDT8;
    cam.precision = 1e-6f;
    std::uniform_real_distribution<float> UX(-6.f, 6.f), UZ(0.05f, 8.f), UP(0.f, 960.f);
    for (int i = 0; i < 2000000; i++) {
        const float X = UX(rng), Y = UX(rng), Z = (i & 7) ? UZ(rng) : UX(rng);
        float u0, v0, u1, v1;
        probe_kb8_project(prm, X, Y, Z, &u0, &v0);
        mam::cam::kb8_project_f(cam, X, Y, Z, &u1, &v1);
        if (bits(u0) != bits(u1) || bits(v0) != bits(v1)) bad_proj++;
        const float px = UP(rng), py = UP(rng);
        float r0[3], r1[3];
        probe_kb8_unproject(prm, cam.precision, px, py, r0);
        mam::cam::kb8_unproject_f(cam, px, py, r1);
        if (bits(r0[0]) != bits(r1[0]) || bits(r0[1]) != bits(r1[1]) || bits(r0[2]) != bits(r1[2])) bad_unproj++;
    }
    const bool ok = !bad_atan && !bad_atan2 && !bad_tan && !bad_proj && !bad_unproj;
    printf("%s atanf %llu/%llu atan2f %llu tanf %llu kb8_project %llu kb8_unproject %llu\n", ok ? "OK" : "FAIL",
           bad_atan, n, bad_atan2, bad_tan, bad_proj, bad_unproj);
    return ok ? 0 : 1;
}
