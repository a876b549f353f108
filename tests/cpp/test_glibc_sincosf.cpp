// Pins the rBRIEF steering trig (ORBextractor.cc:111: sin/cos of a float under `using namespace std`, fused by
// g++ into sincosf) to THIS container's glibc 2.35 libm, the reference image's libm (ros:humble = Ubuntu 22.04).
// Over every float in [0, 2*pi] (or every stride-th one): libm sincosf / sinf / cosf vs
//   - the oracle's restatement (oracle_sincos_policy, policy 0 = FMA build; policy MAM_FP_TRIG_SSE2 = SSE2 build)
//   - the device restatement compiled for the host (det_math.hpp glibc_sincosf<true/false>).
// Prints "OK <n> fma_mismatch 0 sse2_mismatch k" and exits 0 when the host libm's own ifunc choice is matched exactly
// by both restatements.
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>

#include "../../include/mam_orb.h"
#include "../../mam3slam_amd/csrc/det_math.hpp"

extern "C" void oracle_sincos_policy(int fp_policy, float a, float* s, float* c);

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
    const uint32_t stride = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 10) : 1;
    // libm entry points through dlsym: no compiler builtin folding, the ifunc resolves as in the reference process
    void* m = dlopen("libm.so.6", RTLD_NOW);
    auto lsincosf = (void (*)(float, float*, float*))dlsym(m, "sincosf");
    auto lsinf = (float (*)(float))dlsym(m, "sinf");
    auto lcosf = (float (*)(float))dlsym(m, "cosf");
    if (!lsincosf || !lsinf || !lcosf) { printf("FAIL dlsym\n"); return 2; }
    const uint32_t hi = bits(6.2831855f) + 64;   // a little past 2*pi (the float product may round up)
    unsigned long long n = 0, bad_fma = 0, bad_dev = 0, bad_sse2 = 0, bad_sc = 0;
    for (uint32_t u = 0; u <= hi; u += stride) {
        float x;
        memcpy(&x, &u, 4);
        float s, c, so, co, sd, cd, s2, c2, ss2, cs2;
        lsincosf(x, &s, &c);
        if (bits(lsinf(x)) != bits(s) || bits(lcosf(x)) != bits(c)) bad_sc++;
        oracle_sincos_policy(0, x, &so, &co);
        mam::glibc_sincosf<true>(x, &sd, &cd);
        oracle_sincos_policy(MAM_FP_TRIG_SSE2, x, &s2, &c2);
        mam::glibc_sincosf<false>(x, &ss2, &cs2);
        if (bits(so) != bits(s) || bits(co) != bits(c)) bad_fma++;
        if (bits(sd) != bits(so) || bits(cd) != bits(co) || bits(ss2) != bits(s2) || bits(cs2) != bits(c2)) bad_dev++;
        if (bits(s2) != bits(s) || bits(c2) != bits(c)) bad_sse2++;
        n++;
    }
    printf("%s %llu fma_mismatch %llu device_vs_oracle %llu sincosf_vs_sinf_cosf %llu sse2_mismatch %llu\n",
           (bad_fma || bad_dev || bad_sc) ? "FAIL" : "OK", n, bad_fma, bad_dev, bad_sc, bad_sse2);
    return (bad_fma || bad_dev || bad_sc) ? 1 : 0;
}
