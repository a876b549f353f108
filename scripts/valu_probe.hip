// Issue cost and dependent latency of the FP64 VALU forms the LDL^T's pivot chain uses, one wave, clock64 around
// unrolled inline-asm sequences (nothing for the compiler to fold). Prints cycles per instruction.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/valu_probe scripts/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 64
#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))
__global__ void probe(double* out, long long* cyc, const double* in) {
    const int lane = threadIdx.x;
    double a0 = in[lane], a1 = in[lane + 1], a2 = in[lane + 2], a3 = in[lane + 3];
    double a4 = in[lane + 4], a5 = in[lane + 5], a6 = in[lane + 6], a7 = in[lane + 7];
    const double m = in[100], s = in[101];
    float f0 = (float)a0, fm = (float)m;
    long long t0, t1;
    int k = 0;
#define TIME(body)                                              \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
    t0 = clock64();                                             \
    body;                                                       \
    asm volatile("s_nop 0" ::: "memory");                       \
    t1 = clock64();                                             \
    cyc[k++] = t1 - t0;
    // 0 dependent v_fma_f64
    TIME(REP64(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a0) : "v"(m), "v"(s));) asm volatile("" ::"v"(a0)))
    // 1 two independent chains
    TIME(REP8(REP8(asm volatile("v_fma_f64 %0, %0, %2, %3\n\tv_fma_f64 %1, %1, %2, %3" : "+v"(a0), "+v"(a1) : "v"(m), "v"(s));) ))
    // 2 four chains (per 4 instrs)
    TIME(REP8(REP8(asm volatile("v_fma_f64 %0, %0, %4, %5\n\tv_fma_f64 %1, %1, %4, %5\n\tv_fma_f64 %2, %2, %4, %5\n\tv_fma_f64 %3, %3, %4, %5" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(m), "v"(s));)))
    // 3 eight chains
    TIME(REP8(REP8(asm volatile("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\tv_fma_f64 %3, %3, %8, %9\n\tv_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\tv_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(m), "v"(s));)))
    // 4 dependent v_mul_f64
    TIME(REP64(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a1) : "v"(m));))
    // 5 dependent v_rcp_f64
    TIME(REP64(asm volatile("v_rcp_f64 %0, %0" : "+v"(a2));))
    // 6 dependent v_mov_b64_dpp row_newbcast (with the 2 wait states)
    TIME(REP64(asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(a3));))
    // 7 dependent v_fmac_f64_dpp through the accumulator
    TIME(REP64(asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(a4) : "v"(m), "v"(s));))
    // 8 dependent v_fma_f32
    TIME(REP64(asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f0) : "v"(fm));))
    // 9 independent v_fmac_f64_dpp, 8 accumulators (per instr)
    TIME(REP8(asm volatile("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\tv_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(m), "v"(s));))
    // 10 dependent fma chain where the consumer reads the result as a DPP source (mov_dpp then fma), per pair
    TIME(REP64(asm volatile("v_fma_f64 %0, %0, %1, %2\n\ts_nop 1\n\tv_mov_b64_dpp %0, %0 row_newbcast:2 row_mask:0xf bank_mask:0xf" : "+v"(a5) : "v"(m), "v"(s));))
    // 11 ds_read_b64 -> v_fma_f64 -> ds_write_b64 round trip (LDS), per iteration
    __shared__ double sh[64];
    sh[lane] = a6;
    __syncthreads();
    TIME(for (int i = 0; i < N; i++) { double v = sh[lane]; asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v) : "v"(m), "v"(s)); sh[lane] = v; })
    double acc = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (double)f0 + sh[lane ^ 1];
    out[lane] = acc;
}
int main() {
    double *o, *in;
    long long* cy;
    hipMalloc(&o, 64 * sizeof(double));
    hipMalloc(&in, 128 * sizeof(double));
    double h_in[128];
    for (int i = 0; i < 128; i++) h_in[i] = 1.0 + i * 1e-3;
    h_in[100] = 0.999999;
    h_in[101] = 1e-9;
    hipMemcpy(in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
    hipMalloc(&cy, 16 * sizeof(long long));
    const char* names[] = {"fma_f64 dependent", "fma_f64 2 chains", "fma_f64 4 chains", "fma_f64 8 chains",
                           "mul_f64 dependent", "rcp_f64 dependent", "mov_b64_dpp dependent (+nop1)",
                           "fmac_f64_dpp dependent (acc)", "fma_f32 dependent", "fmac_f64_dpp 8 independent",
                           "fma_f64 -> mov_b64_dpp pair", "lds read-fma-write round trip"};
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, o, cy, in);
        (void)hipDeviceSynchronize();
        long long h[16];
        (void)hipMemcpy(h, cy, sizeof(h), hipMemcpyDeviceToHost);
        if (rep == 2)
            for (int i = 0; i < 12; i++) printf("%-32s %6lld cycles / 64 = %6.2f\n", names[i], h[i], h[i] / 64.0);
    }
    return 0;
}
