// pose.hip — gfx950 Optimizer::PoseOptimization (include/mam_pose.h): the whole 4-round Levenberg-Marquardt of one
// frame's pose in ONE workgroup, batched over frames (one workgroup per frame), FP64 throughout.
//
// Reference: src/Optimizer.cc:814-1115 with g2o's Levenberg (core/optimization_algorithm_levenberg.cpp:61-169),
// BlockSolver_6_3 + LinearSolverDense (Eigen LDLT, solvers/linear_solver_dense.h:65-118), EdgeSE3ProjectXYZOnlyPose
// (src/OptimizableTypes.cpp:49-63) and RobustKernelHuber (core/robust_kernel_impl.cpp:76-91).
//
// Layout: the frame's edges are staged in LDS as float SoA (obs x/y, Xw, invSigma2; the reference's float inputs,
// widened to double where used) next to each edge's last error (2 doubles, the stale-after-rejected-trial value
// g2o's chi2() reads) and its level (0 active, 1 outlier). Every pass deals the edges to the PT threads; the
// per-thread partial sums (robust chi2, or the 21 upper entries of H plus b) are reduced by a fixed DPP pattern
// per wave and a fixed wave order, so every thread ends with the same bits and runs the LM control flow; the 6x6
// pivoted LDL^T and the SE3 update run redundantly in every wave when there is one wave per SIMD, on wave 0 with an LDS
// broadcast when there are more (no host round trip, block-uniform branches).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>

#include "../../include/mam_pose.h"
#include "camera.hpp"
#include "runtime.hpp"
#include "se3.hpp"

namespace mam {
namespace pose {

// threads per frame, per camera model: Pinhole 512 (two waves per SIMD hide the edge passes' FP64 latency; the serial
// LM step then runs on wave 0 only: batch of 16 c2 frames 0.423 -> 0.368 ms), KannalaBrandt8 256 (its projection and
// Jacobian spill at 512's register budget); 1024 spills either way
#ifndef MAM_POSE_THREADS
#define MAM_POSE_THREADS 512
#endif
#ifndef MAM_POSE_THREADS_KB8
#define MAM_POSE_THREADS_KB8 256
#endif
template <bool KB8>
struct Cfg {
    static constexpr int PT = KB8 ? MAM_POSE_THREADS_KB8 : MAM_POSE_THREADS;
    static constexpr int NW = PT / 64;
};
#ifndef MAM_POSE_BUILD_UNROLL
#define MAM_POSE_BUILD_UNROLL 2
#endif
// 1: every wave runs the serial LM step itself (no wave-0 solve + LDS broadcast); an experiment switch
#ifndef MAM_POSE_STEP_ALL_WAVES
#define MAM_POSE_STEP_ALL_WAVES 0
#endif
#ifndef MAM_POSE_CHI_UNROLL
#define MAM_POSE_CHI_UNROLL 2
#endif
#define MAM_POSE_PRAGMA_(x) _Pragma(#x)
#define MAM_POSE_PRAGMA(x) MAM_POSE_PRAGMA_(x)
constexpr int NRED = 27;       // 21 upper entries of H + 6 of b

#ifdef MAM_POSE_PROFILE
// phase cycles (thread 0 of every workgroup): 0 build pass + sums, 1 LDL^T solve, 2 exp * T, 3 trial pass + sum,
// 4 LM control, 5 trials, 6 build passes
__device__ unsigned long long g_pprof[16];
// thread 0 accumulates in LDS (a global atomic per probe would put its memory latency into the next barrier) and
// flushes once at the end of the workgroup
__shared__ unsigned long long s_pprof[16];
#define PPROF(k, t0)                                                                    \
    do {                                                                                \
        const long long tn_ = clock64();                                               \
        if (threadIdx.x == 0) s_pprof[k] += (unsigned long long)(tn_ - (t0));           \
        (t0) = tn_;                                                                     \
    } while (0)
#else
#define PPROF(k, t0) \
    do {             \
    } while (0)
#endif

struct Args {
    int nframes;
    const mam_pose* tcw;
    mam_camera cam;
    const mam_pose_edge* edges;
    int stride;
    const int32_t* n_edges;
    uint8_t* outlier;
    mam_pose_result* res;
    int cap;                   // edges the LDS carve holds
};

__host__ __device__ inline size_t a16(size_t b) { return (b + 15) & ~(size_t)15; }
// floats: 6 per edge (SoA), errors: 2 doubles per edge, level: 1 byte per edge
__host__ __device__ inline size_t lds_bytes(int cap) {
    return a16((size_t)cap * 16) + 6 * a16((size_t)cap * 4) + a16((size_t)cap);
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, CTRL, 0xF, 0xF, false),
                            __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xF, 0xF, false));
}

// 1 / a as v_rcp_f64 + two Newton steps (the fdiv lowering without its range scaling: |a| stays far inside the
// normal range here); within an ulp of the quotient, half the dependent instructions
__device__ __forceinline__ double rcp_nr(double a) {
    double r = __builtin_amdgcn_rcp(a);
    double e = fma(-a, r, 1.0);
    r = fma(r, e, r);
    e = fma(-a, r, 1.0);
    return fma(r, e, r);
}

// Wave sum with a fixed DPP pattern (quad perms, row shifts, row broadcasts); the total lands in lane 63.
__device__ __forceinline__ double wave_sum63(double v) {
    v += dpp_d<0xb1>(v);    // quad_perm [1,0,3,2]
    v += dpp_d<0x4e>(v);    // quad_perm [2,3,0,1]
    v += dpp_d<0x114>(v);   // row_shr:4
    v += dpp_d<0x118>(v);   // row_shr:8
    v += dpp_d<0x142>(v);   // row_bcast:15
    v += dpp_d<0x143>(v);   // row_bcast:31
    return v;
}

__device__ __forceinline__ double lane63(double v) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63),
                            __builtin_amdgcn_readlane(__double2loint(v), 63));
}

// 4 Q wave sums at once, reduce-scatter style: the xor-32 and xor-16 steps exchange only the half of the values the
// lane keeps, then xor 8 .. 1 on the Q left; lane group g = lane >> 4 ends with sums [g Q, g Q + Q) (fixed pattern:
// the bits do not depend on timing) — 7 Q shuffles instead of a full reduction per value
// a(l) + a(l ^ 32) on lanes 0-31, b(l ^ 32) + b(l) on lanes 32-63: one v_permlane32_swap per dword (gfx950), no LDS
__device__ __forceinline__ double swap32_sum(double a, double b) {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
// the same across rows of 16: a on even rows, b on odd rows
__device__ __forceinline__ double swap16_sum(double a, double b) {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}

template <int Q>
__device__ __forceinline__ void wave_sum_scatter4(const double (&v)[4 * Q], double (&out)[Q]) {
#ifndef MAM_POSE_SHFL
    // lanes swap through v_permlane{32,16}_swap, then a symmetric DPP butterfly inside each row (every lane of the row
    // ends with the same bits: each step adds the same two partials in either order)
    double h[2 * Q];
#pragma unroll
    for (int i = 0; i < 2 * Q; i++) h[i] = swap32_sum(v[i], v[2 * Q + i]);
#pragma unroll
    for (int i = 0; i < Q; i++) out[i] = swap16_sum(h[i], h[Q + i]);
#pragma unroll
    for (int i = 0; i < Q; i++) out[i] += dpp_d<0xb1>(out[i]);    // quad_perm [1,0,3,2]
#pragma unroll
    for (int i = 0; i < Q; i++) out[i] += dpp_d<0x4e>(out[i]);    // quad_perm [2,3,0,1]
#pragma unroll
    for (int i = 0; i < Q; i++) out[i] += dpp_d<0x141>(out[i]);   // row_half_mirror
#pragma unroll
    for (int i = 0; i < Q; i++) out[i] += dpp_d<0x140>(out[i]);   // row_mirror
#else
    const int lane = threadIdx.x & 63;
    const bool b5 = (lane & 32) != 0, b4 = (lane & 16) != 0;
    double h[2 * Q];
#pragma unroll
    for (int i = 0; i < 2 * Q; i++) {
        const double send = b5 ? v[i] : v[2 * Q + i];
        const double keep = b5 ? v[2 * Q + i] : v[i];
        h[i] = keep + __shfl_xor(send, 32, 64);
    }
#pragma unroll
    for (int i = 0; i < Q; i++) {
        const double send = b4 ? h[i] : h[Q + i];
        const double keep = b4 ? h[Q + i] : h[i];
        out[i] = keep + __shfl_xor(send, 16, 64);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1)
#pragma unroll
        for (int i = 0; i < Q; i++) out[i] += __shfl_xor(out[i], o, 64);
#endif
}

// Block sum of N per-thread values into out[0..N) (LDS; waves summed in order 0..NW-1, a fixed pattern inside a
// wave, so the bits do not depend on timing). Ends with a barrier: out[] is readable by every thread.
template <int N, int NW>
__device__ __forceinline__ void block_sum(const double (&v)[N], double* scr, double* out) {
    const int w = threadIdx.x >> 6;
#ifdef MAM_POSE_PROFILE
    long long tq = clock64();
#endif
    if constexpr (N % 4 == 0 && N >= 8) {
        constexpr int Q = N / 4;
        double tot[Q];
        wave_sum_scatter4<Q>(v, tot);
        const int lane = threadIdx.x & 63, il = lane & 15;
        double val = 0.0;
#pragma unroll
        for (int i = 0; i < Q; i++) val = il == i ? tot[i] : val;
        if (il < Q) scr[w * N + Q * (lane >> 4) + il] = val;
        PPROF(8, tq);
    } else {
#pragma unroll
        for (int k = 0; k < N; k++) {
            const double s = lane63(wave_sum63(v[k]));
            if ((threadIdx.x & 63) == 0) scr[w * N + k] = s;
        }
    }
    __syncthreads();
    if (N > 1) PPROF(9, tq);
    if (threadIdx.x < N) {
        double s = scr[threadIdx.x];
#pragma unroll
        for (int q = 1; q < NW; q++) s += scr[q * N + threadIdx.x];
        out[threadIdx.x] = s;
    }
    __syncthreads();
    if (N > 1) PPROF(10, tq);
}

struct Edges {
    const float *ox, *oy, *X, *Y, *Z, *w;
    double* err;
    uint8_t* level;
    int n;
};

// T as a rotation matrix + translation (Eigen QuaternionBase::toRotationMatrix), once per pass: T.map(Xw) is then
// 9 FMAs per edge instead of the quaternion form's 30 instructions (within a few ulp of it; the 1e-4 pose parity)
struct Rt {
    double r[9], t[3];
};
__device__ __forceinline__ Rt make_rt(const double T[7]) {
    const double x = T[0], y = T[1], z = T[2], w = T[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    Rt m;
    m.r[0] = 1 - (tyy + tzz); m.r[1] = txy - twz;       m.r[2] = txz + twy;
    m.r[3] = txy + twz;       m.r[4] = 1 - (txx + tzz); m.r[5] = tyz - twx;
    m.r[6] = txz - twy;       m.r[7] = tyz + twx;       m.r[8] = 1 - (txx + tyy);
    m.t[0] = T[4]; m.t[1] = T[5]; m.t[2] = T[6];
    return m;
}
__device__ __forceinline__ void map_rt(const Rt& m, const double X[3], double o[3]) {
#pragma unroll
    for (int r = 0; r < 3; r++) o[r] = fma(m.r[3 * r], X[0], fma(m.r[3 * r + 1], X[1], fma(m.r[3 * r + 2], X[2], m.t[r])));
}

// EdgeSE3ProjectXYZOnlyPose::computeError: obs - Pinhole::project(T.map(Xw)); returns chi2 = e^T (w I) e
template <bool KB8>
__device__ __forceinline__ double edge_error(const Edges& E, int i, const Rt& T, const mam_camera& c,
                                             double* e0o, double* e1o) {
    const double Xw[3] = {(double)E.X[i], (double)E.Y[i], (double)E.Z[i]};
    double Xc[3];
    map_rt(T, Xw, Xc);
    double u, v;
    if (KB8) {
        cam::project_d(c, Xc, &u, &v);   // KannalaBrandt8::project(Vector3d)
    } else {
        const double iz = rcp_nr(Xc[2]);   // one reciprocal, two products (within an ulp of fx * x / z)
        u = (double)c.fx * Xc[0] * iz + (double)c.cx;
        v = (double)c.fy * Xc[1] * iz + (double)c.cy;
    }
    const double e0 = (double)E.ox[i] - u, e1 = (double)E.oy[i] - v;
    *e0o = e0;
    *e1o = e1;
    const double w = (double)E.w[i];
    return e0 * (w * e0) + e1 * (w * e1);
}

// O = SE3Quat::exp(u) * T (VertexSE3Expmap::oplusImpl, types/se3quat.h) for the LM step, on its serial critical path:
// the rotation's quaternion straight from the half angle, (sin(θ/2) / θ · ω, cos(θ/2)) — what Quaterniond(R(ω))
// gives up to rounding, also in g2o's θ < 1e-5 branch, whose I + Ω + Ω² agrees with the rotation to O(θ⁴) after the
// normalisation — and V's Rodrigues coefficients (1 - cos θ) / θ², (θ - sin θ) / θ³ as their Taylor series below
// θ = 0.25 (truncation below 1e-18; one sincos pair above), V = I + Ω + Ω² below θ = 1e-5 as g2o has it.
__device__ __forceinline__ void exp_mul_step(const double u[6], const double T[7], double O[7]) {
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double th2 = w0 * w0 + w1 * w1 + w2 * w2;
    const double th = sqrt(th2);
    double sh, ch, b, c;   // sin(θ/2) / θ, cos(θ/2), (1 - cos θ) / θ², (θ - sin θ) / θ³
    // θ is the same in every lane: a scalar branch, so the sincos path is not if-converted into the series path
    if (__builtin_amdgcn_readfirstlane(th < 0.25 ? 1 : 0)) {
        const double x = 0.25 * th2;   // (θ/2)²
        double s = fma(x, 1.0 / 6227020800.0, -1.0 / 39916800.0);
        s = fma(x, s, 1.0 / 362880.0);
        s = fma(x, s, -1.0 / 5040.0);
        s = fma(x, s, 1.0 / 120.0);
        s = fma(x, s, -1.0 / 6.0);
        s = fma(x, s, 1.0);
        sh = 0.5 * s;
        double k = fma(x, 1.0 / 479001600.0, -1.0 / 3628800.0);
        k = fma(x, k, 1.0 / 40320.0);
        k = fma(x, k, -1.0 / 720.0);
        k = fma(x, k, 1.0 / 24.0);
        k = fma(x, k, -0.5);
        ch = fma(x, k, 1.0);
        double bb = fma(th2, -1.0 / 20922789888000.0, 1.0 / 87178291200.0);
        bb = fma(th2, bb, -1.0 / 479001600.0);
        bb = fma(th2, bb, 1.0 / 3628800.0);
        bb = fma(th2, bb, -1.0 / 40320.0);
        bb = fma(th2, bb, 1.0 / 720.0);
        bb = fma(th2, bb, -1.0 / 24.0);
        b = fma(th2, bb, 0.5);
        double cc = fma(th2, -1.0 / 355687428096000.0, 1.0 / 1307674368000.0);
        cc = fma(th2, cc, -1.0 / 6227020800.0);
        cc = fma(th2, cc, 1.0 / 39916800.0);
        cc = fma(th2, cc, -1.0 / 362880.0);
        cc = fma(th2, cc, 1.0 / 5040.0);
        cc = fma(th2, cc, -1.0 / 120.0);
        c = fma(th2, cc, 1.0 / 6.0);
    } else {
        // an opaque copy of θ: the sincos pair cannot be speculated above the branch onto the common path
        double thv = th;
        asm volatile("" : "+v"(thv));
        double sn, cs, s2, c2;
        sincos(thv, &sn, &cs);
        sincos(0.5 * thv, &s2, &c2);
        const double it = 1.0 / thv;
        sh = s2 * it;
        ch = c2;
        b = (1 - cs) * (it * it);
        c = (thv - sn) * (it * it * it);
    }
    if (th < 0.00001) { b = 1.0; c = 1.0; }   // g2o's small-angle V = I + Ω + Ω²
    const double qe[4] = {sh * w0, sh * w1, sh * w2, ch};
    // V u_t = u_t + b (ω × u_t) + c (ω × (ω × u_t))
    const double t0 = u[3], t1 = u[4], t2 = u[5];
    const double x0 = w1 * t2 - w2 * t1, x1 = w2 * t0 - w0 * t2, x2 = w0 * t1 - w1 * t0;
    const double y0 = w1 * x2 - w2 * x1, y1 = w2 * x0 - w0 * x2, y2 = w0 * x1 - w1 * x0;
    const double te[3] = {fma(c, y0, fma(b, x0, t0)), fma(c, y1, fma(b, x1, t1)), fma(c, y2, fma(b, x2, t2))};
    double rt[3];
    se3::quat_rotate(qe, T + 4, rt);
    double q[4];
    q[3] = qe[3] * T[3] - qe[0] * T[0] - qe[1] * T[1] - qe[2] * T[2];
    q[0] = qe[3] * T[0] + qe[0] * T[3] + qe[1] * T[2] - qe[2] * T[1];
    q[1] = qe[3] * T[1] + qe[1] * T[3] + qe[2] * T[0] - qe[0] * T[2];
    q[2] = qe[3] * T[2] + qe[2] * T[3] + qe[0] * T[1] - qe[1] * T[0];
    if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
    const double r = rcp_nr(sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]));
    O[0] = q[0] * r; O[1] = q[1] * r; O[2] = q[2] * r; O[3] = q[3] * r;
    O[4] = te[0] + rt[0]; O[5] = te[1] + rt[1]; O[6] = te[2] + rt[2];
}

// RobustKernelHuber::robustify (core/robust_kernel_impl.cpp:76-91) with sqrt(e) and delta / sqrt(e) from one
// v_rsq_f64 + two Newton steps (within a few ulp of the sqrt and the quotient; the 1e-4 pose parity)
__device__ __forceinline__ void rho_of(double chi, bool robust, double delta, double* r0, double* r1) {
    const double dsqr = delta * delta;
    if (!robust || chi <= dsqr) { *r0 = chi; *r1 = 1.0; }
    else {
        double y = __builtin_amdgcn_rsq(chi);
        const double h = 0.5 * chi;
        y = y * fma(-h * y, y, 1.5);
        y = y * fma(-h * y, y, 1.5);
        const double sq = chi * y;
        *r0 = 2 * sq * delta - dsqr;
        *r1 = delta * y;
    }
}


// computeActiveErrors at T (errors stored) + activeRobustChi2
template <bool KB8>
__device__ double active_chi(const Edges& E, const double T[7], const mam_camera& c, bool robust, double delta,
                             double* scr) {
    constexpr int PT = Cfg<KB8>::PT, NW = Cfg<KB8>::NW;
    double acc[1] = {0.0};
    const Rt Rm = make_rt(T);
    MAM_POSE_PRAGMA(unroll MAM_POSE_CHI_UNROLL)
    for (int i = threadIdx.x; i < E.n; i += PT) {
        if (E.level[i]) continue;
        double e0, e1;
        const double chi = edge_error<KB8>(E, i, Rm, c, &e0, &e1);
        E.err[2 * i] = e0;
        E.err[2 * i + 1] = e1;
        double r0, r1;
        rho_of(chi, robust, delta, &r0, &r1);
        acc[0] += r0;
    }
    block_sum<1, NW>(acc, scr, scr + NW * (NRED + 1));
    return scr[NW * (NRED + 1)];
}

// One pass: computeActiveErrors + activeRobustChi2 + buildSystem (BaseUnaryEdge::constructQuadraticForm,
// base_unary_edge.hpp:43-71). H upper (row-major i <= j, 21) then b (6) in red[0..26]; returns the chi.
template <bool KB8>
__device__ double build_system(const Edges& E, const double T[7], const mam_camera& c, bool robust, double delta,
                               double* scr, double* red) {
    constexpr int PT = Cfg<KB8>::PT, NW = Cfg<KB8>::NW;
    double acc[NRED + 1];
#pragma unroll
    for (int k = 0; k <= NRED; k++) acc[k] = 0.0;
    const Rt Rm = make_rt(T);
#ifdef MAM_POSE_PROFILE
    long long tb = clock64();
#endif
    // two edges per iteration: their dependency chains (map, divisions, robust weight, Jacobian, sums) interleave —
    // one wave per SIMD has nothing else to hide the FP64 latency with
    MAM_POSE_PRAGMA(unroll MAM_POSE_BUILD_UNROLL)
    for (int i = threadIdx.x; i < E.n; i += PT) {
        if (E.level[i]) continue;
        const double Xw[3] = {(double)E.X[i], (double)E.Y[i], (double)E.Z[i]};
        double Xc[3];
        map_rt(Rm, Xw, Xc);
        const double x = Xc[0], y = Xc[1], z = Xc[2];
        constexpr bool kb8 = KB8;
        double u, v, iz = 0.0, fxz = 0.0, fyz = 0.0;
        if (kb8) {
            cam::project_d(c, Xc, &u, &v);
        } else {
            // Pinhole with one reciprocal of z for the projection and the Jacobian (six divisions before; the
            // products are within an ulp of the quotients, inside the 1e-4 pose parity)
            iz = rcp_nr(z);
            fxz = (double)c.fx * x * iz;
            fyz = (double)c.fy * y * iz;
            u = fxz + (double)c.cx;
            v = fyz + (double)c.cy;
        }
        const double e0 = (double)E.ox[i] - u, e1 = (double)E.oy[i] - v;
        E.err[2 * i] = e0;
        E.err[2 * i + 1] = e1;
        const double w = (double)E.w[i];
        const double chi = e0 * (w * e0) + e1 * (w * e1);
        double r0, r1;
        rho_of(chi, robust, delta, &r0, &r1);
        acc[NRED] += r0;
        // _jacobianOplusXi = -projectJac(Xc) * SE3deriv (OptimizableTypes.cpp:49-63)
        double J[6];
        if (kb8) {
            cam::project_jac_d(c, Xc, J);   // KannalaBrandt8::projectJac (KannalaBrandt8.cpp:145-175)
#pragma unroll
            for (int k = 0; k < 6; k++) J[k] = -J[k];
        } else {
            const double fx = c.fx, fy = c.fy;
            J[0] = -(fx * iz); J[1] = -0.0; J[2] = fxz * iz;
            J[3] = -0.0; J[4] = -(fy * iz); J[5] = fyz * iz;
        }
        double A[12];
        if (kb8) {
            const double D[18] = {0.0, z, -y, 1.0, 0.0, 0.0, -z, 0.0, x, 0.0, 1.0, 0.0, y, -x, 0.0, 0.0, 0.0, 1.0};
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int k = 0; k < 6; k++)
                    A[6 * r + k] = J[3 * r] * D[k] + J[3 * r + 1] * D[6 + k] + J[3 * r + 2] * D[12 + k];
        } else {
            // the same product with Pinhole's zero Jacobian entries and SE3deriv's zeros / ones folded: every
            // non-zero entry gets the same operations (a product with an exact zero adds a signed zero, which leaves
            // a non-zero sum unchanged); the entries that are exactly zero become +0
            const double J0 = J[0], J2 = J[2], J4 = J[4], J5 = J[5];
            A[0] = J2 * y;          A[1] = J0 * z + J2 * -x; A[2] = J0 * -y;
            A[3] = J0;              A[4] = 0.0;              A[5] = J2;
            A[6] = J4 * -z + J5 * y; A[7] = J5 * -x;         A[8] = J4 * x;
            A[9] = 0.0;             A[10] = J4;              A[11] = J5;
        }
        const double o0 = -(w * e0) * r1, o1 = -(w * e1) * r1;
        const double wo = r1 * w;
        double wA[12];   // A * wo once per entry: (A[a] * wo) * A[b] is the same product as before
#pragma unroll
        for (int k = 0; k < 12; k++) wA[k] = A[k] * wo;
        // H and b as FMA chains; Pinhole's structural zeros (A[4], A[9]) skipped (the loops unroll, so the tests fold)
        int q = 0;
#pragma unroll
        for (int a = 0; a < 6; a++)
#pragma unroll
            for (int b = a; b < 6; b++) {
                double h = acc[q];
                if (kb8 || (a != 3 && b != 3)) h = fma(wA[6 + a], A[6 + b], h);
                if (kb8 || (a != 4 && b != 4)) h = fma(wA[a], A[b], h);
                acc[q++] = h;
            }
#pragma unroll
        for (int a = 0; a < 6; a++) {
            double g = acc[21 + a];
            if (kb8 || a != 3) g = fma(A[6 + a], o1, g);
            if (kb8 || a != 4) g = fma(A[a], o0, g);
            acc[21 + a] = g;
        }
    }
    PPROF(7, tb);   // the edge loop alone (thread 0's view)
    block_sum<NRED + 1, NW>(acc, scr, red);
    return red[NRED];
}

// (H + lambda I) x = b, 6x6: Eigen 3.4.0 LDLT<MatrixXd, Lower>'s left-looking LDL^T and solve
// (oracle/pose_oracle.cpp eigen_ldlt_solve) without its diagonal pivoting, returning isPositive() (no negative
// pivot). H = J^T W J is positive semi-definite (Huber weights are positive) and lambda > 0, so the unpivoted LDL^T is
// as stable as the pivoted one; only the rounding differs (within the 1e-4 pose parity). Pivoting cost three times the
// instructions of the factorization itself in row / column exchanges and the inverse permutation (a runtime-indexed
// private array would live in scratch memory). Dot products as FMA chains, one reciprocal per pivot.
__device__ bool ldlt6(const double* red, double lambda, double x[6]) {
    double m[36];   // lower triangle used
    {
        int q = 0;
#pragma unroll
        for (int a = 0; a < 6; a++)
#pragma unroll
            for (int b = a; b < 6; b++) m[6 * b + a] = red[q++];
#pragma unroll
        for (int j = 0; j < 6; j++) m[7 * j] += lambda;
    }
    double d[6];
#pragma unroll
    for (int j = 0; j < 6; j++) d[j] = red[21 + j];
    double rd[6];
    bool neg = false;   // a negative pivot: Eigen's sign ends NegativeSemiDef or Indefinite
#pragma unroll
    for (int k = 0; k < 6; k++) {
        if (k > 0) {
            double temp[6];
#pragma unroll
            for (int j = 0; j < k; j++) temp[j] = m[7 * j] * m[6 * k + j];
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < k; j++) s = fma(m[6 * k + j], temp[j], s);
            m[7 * k] -= s;
#pragma unroll
            for (int i = k + 1; i < 6; i++) {
                double t = 0.0;
#pragma unroll
                for (int j = 0; j < k; j++) t = fma(m[6 * i + j], temp[j], t);
                m[6 * i + k] -= t;
            }
        }
        const double akk = m[7 * k];
        const double rk = rcp_nr(akk);
        rd[k] = rk;
        const double rs = fabs(akk) > 0.0 ? rk : 1.0;   // a zero pivot leaves its column as it is
#pragma unroll
        for (int i = k + 1; i < 6; i++) m[6 * i + k] *= rs;
        neg = neg || akk < 0.0;
    }
#pragma unroll
    for (int k = 0; k < 6; k++)
#pragma unroll
        for (int i = k + 1; i < 6; i++) d[i] = fma(-m[6 * i + k], d[k], d[i]);
    const double tol = 2.2250738585072014e-308;   // numeric_limits<double>::min()
#pragma unroll
    for (int i = 0; i < 6; i++) d[i] = fabs(m[7 * i]) > tol ? d[i] * rd[i] : 0.0;
#pragma unroll
    for (int k = 5; k >= 0; k--)
#pragma unroll
        for (int i = 0; i < k; i++) d[i] = fma(-m[6 * k + i], d[k], d[i]);
#pragma unroll
    for (int j = 0; j < 6; j++) x[j] = d[j];
    return !neg;
}


// SparseOptimizer::optimize(10) on the single pose vertex; T is updated in place. Returns the iterations run.
template <bool KB8>
__device__ int optimize(const Edges& E, double T[7], const mam_camera& c, bool robust, double delta, double* scr,
                        int* trials) {
    constexpr int PT = Cfg<KB8>::PT, NW = Cfg<KB8>::NW;
    // initializeOptimization(0): no level-0 edge -> optimize() returns -1 before the loop
    __shared__ int s_any;
    if (threadIdx.x == 0) s_any = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < E.n; i += PT)
        if (!E.level[i]) { s_any = 1; break; }
    __syncthreads();
    const bool any = s_any != 0;
    __syncthreads();
    if (!any) return 0;
    double lambda = 0.0, ni = 2.0;
    int nBad = 0, its = 0;
    bool ok = true;
    for (int it = 0; it < 10 && ok; it++) {
        double* red = scr + NW * (NRED + 1) + 8;   // H upper, b, chi (LDS)
#ifdef MAM_POSE_PROFILE
        long long tp = clock64();
#endif
        double currentChi = build_system<KB8>(E, T, c, robust, delta, scr, red);
        PPROF(0, tp);
#ifdef MAM_POSE_PROFILE
        if (threadIdx.x == 0) s_pprof[6] += 1ull;
#endif
        const double iniChi = currentChi;
        if (it == 0) {
            double md = 0.0;
            md = fmax(fabs(red[0]), md);    // H(0,0)
            md = fmax(fabs(red[6]), md);    // H(1,1)
            md = fmax(fabs(red[11]), md);   // H(2,2)
            md = fmax(fabs(red[15]), md);   // H(3,3)
            md = fmax(fabs(red[18]), md);   // H(4,4)
            md = fmax(fabs(red[20]), md);   // H(5,5)
            lambda = 1e-5 * md;
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            double x[6];
            PPROF(4, tp);   // LM control since the last pass
            bool ok2;
            double Tn[7];
            if constexpr (NW > 4 && !MAM_POSE_STEP_ALL_WAVES) {
                // more waves than SIMDs: the serial step on wave 0 only (redundant copies would share its SIMD's
                // issue slots), x / Tn / the verdict broadcast through LDS
                __shared__ double s_step[14];
                if (threadIdx.x < 64) {
#ifdef MAM_POSE_PROFILE
                    long long tl = clock64();
#endif
                    ok2 = ldlt6(red, lambda, x);
                    PPROF(11, tl);
                    exp_mul_step(x, T, Tn);
                    PPROF(12, tl);
                    if (threadIdx.x == 0) {
#pragma unroll
                        for (int k = 0; k < 6; k++) s_step[k] = x[k];
#pragma unroll
                        for (int k = 0; k < 7; k++) s_step[6 + k] = Tn[k];
                        s_step[13] = ok2 ? 1.0 : 0.0;
                    }
                }
                __syncthreads();
#pragma unroll
                for (int k = 0; k < 6; k++) x[k] = s_step[k];
#pragma unroll
                for (int k = 0; k < 7; k++) Tn[k] = s_step[6 + k];
                ok2 = s_step[13] != 0.0;
                PPROF(2, tp);
            } else {
                ok2 = ldlt6(red, lambda, x);
                PPROF(1, tp);
                exp_mul_step(x, T, Tn);
                PPROF(2, tp);
            }
            double tempChi = active_chi<KB8>(E, Tn, c, robust, delta, scr);
            PPROF(3, tp);
#ifdef MAM_POSE_PROFILE
            if (threadIdx.x == 0) s_pprof[5] += 1ull;
#endif
            if (!ok2) tempChi = 1.7976931348623157e308;
            rho = currentChi - tempChi;
            double scale = 0.0;
            for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + red[21 + j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && isfinite(tempChi)) {
                double alpha = 1. - pow((2 * rho - 1), 3);
                alpha = fmin(alpha, 2. / 3.);
                lambda *= fmax(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
                for (int k = 0; k < 7; k++) T[k] = Tn[k];
            } else {
                lambda *= ni;
                ni *= 2;
            }
            qmax++;
            (*trials)++;
        } while (rho < 0 && qmax < 10);
        its++;
        if (qmax == 10 || rho == 0) ok = false;
        else {
            if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
            else nBad = 0;
            if (nBad >= 3) ok = false;
        }
    }
    return its;
}

// the camera model is a template parameter: a Pinhole launch carries no KannalaBrandt8 code in its edge loops
template <bool KB8>
__global__ __launch_bounds__(Cfg<KB8>::PT) void k_pose_opt(Args a) {
    constexpr int PT = Cfg<KB8>::PT, NW = Cfg<KB8>::NW;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ double scr[NW * (NRED + 1) + 8 + NRED + 1];   // wave partials | chi sum | H, b, chi sums
    __shared__ int s_nbad;
    const int f = blockIdx.x, t = threadIdx.x;
    const int n = a.n_edges[f];
    mam_pose_result* R = a.res + f;
    if (n < 0 || n > a.cap) {
        if (t == 0) { R->n_inliers = MAM_ERR_CAPACITY; R->rounds = 0; R->iterations = 0; R->lm_trials = 0; }
        return;
    }
#ifdef MAM_POSE_PROFILE
    if (t < 16) s_pprof[t] = 0;
#endif
    uint8_t* p = smem;
    Edges E;
    E.err = reinterpret_cast<double*>(p);      p += a16((size_t)a.cap * 16);
    float* ox = reinterpret_cast<float*>(p);   p += a16((size_t)a.cap * 4);
    float* oy = reinterpret_cast<float*>(p);   p += a16((size_t)a.cap * 4);
    float* X = reinterpret_cast<float*>(p);    p += a16((size_t)a.cap * 4);
    float* Y = reinterpret_cast<float*>(p);    p += a16((size_t)a.cap * 4);
    float* Z = reinterpret_cast<float*>(p);    p += a16((size_t)a.cap * 4);
    float* W = reinterpret_cast<float*>(p);    p += a16((size_t)a.cap * 4);
    E.level = p;
    E.ox = ox; E.oy = oy; E.X = X; E.Y = Y; E.Z = Z; E.w = W;
    E.n = n;
    const mam_pose_edge* ge = a.edges + (size_t)f * a.stride;
    uint8_t* out = a.outlier + (size_t)f * a.stride;
    for (int i = t; i < n; i += PT) {
        const mam_pose_edge e = ge[i];
        ox[i] = e.obs[0]; oy[i] = e.obs[1]; X[i] = e.xw[0]; Y[i] = e.xw[1]; Z[i] = e.xw[2]; W[i] = e.inv_sigma2;
        E.level[i] = 0;
    }
    // SE3Quat(Tcw.unit_quaternion().cast<double>(), translation) (normalised)
    const mam_pose P0 = a.tcw[f];
    double T0[7] = {(double)P0.q[0], (double)P0.q[1], (double)P0.q[2], (double)P0.q[3],
                    (double)P0.t[0], (double)P0.t[1], (double)P0.t[2]};
    se3::normalize_q(T0);
    double T[7];
    for (int k = 0; k < 7; k++) T[k] = T0[k];
    int rounds = 0, its = 0, trials = 0, nBad = 0;
    __syncthreads();
    if (n >= 3) {
        const double delta = (double)(float)sqrt(5.991);   // const float deltaMono = sqrt(5.991) (Optimizer.cc:850)
        bool robust = true;
        for (int it = 0; it < 4; it++) {
            for (int k = 0; k < 7; k++) T[k] = T0[k];   // vSE3->setEstimate(pFrame->GetPose())
            its += optimize<KB8>(E, T, a.cam, robust, delta, scr, &trials);
            rounds++;
            if (t == 0) s_nbad = 0;
            __syncthreads();
            int bad = 0;
            const Rt Rm = make_rt(T);
            for (int i = t; i < n; i += PT) {
                if (E.level[i]) {   // outliers of the last classification: computeError() at the new pose
                    double e0, e1;
                    edge_error<KB8>(E, i, Rm, a.cam, &e0, &e1);
                    E.err[2 * i] = e0;
                    E.err[2 * i + 1] = e1;
                }
                const double e0 = E.err[2 * i], e1 = E.err[2 * i + 1], w = (double)E.w[i];
                const float chi2 = (float)(e0 * (w * e0) + e1 * (w * e1));   // const float chi2 = e->chi2()
                const bool o = chi2 > 5.991f;
                E.level[i] = o ? 1 : 0;
                bad += o ? 1 : 0;
            }
            if (bad) atomicAdd(&s_nbad, bad);
            __syncthreads();
            nBad = s_nbad;
            __syncthreads();
            if (it == 2) robust = false;
            if (n < 10) break;
        }
    }
    for (int i = t; i < n; i += PT) out[i] = E.level[i];
#ifdef MAM_POSE_PROFILE
    __syncthreads();
    if (t < 16) atomicAdd(&g_pprof[t], s_pprof[t]);
#endif
    if (t == 0) {
        R->q[0] = T[0]; R->q[1] = T[1]; R->q[2] = T[2]; R->q[3] = T[3];
        R->t[0] = T[4]; R->t[1] = T[5]; R->t[2] = T[6];
        R->n_inliers = n >= 3 ? n - nBad : 0;
        R->rounds = rounds;
        R->iterations = its;
        R->lm_trials = trials;
    }
}

// ---- the frame side of the call (device-resident tracked frames)
// Optimizer::PoseOptimization's edge list (Optimizer.cc:856-895): one mono edge per keypoint i whose slot holds a
// MapPoint (mvpMapPoints[i] != NULL), in increasing i, observation mvKeysUn[i].pt (= mvKeys: k1 = 0), information
// mvInvLevelSigma2[octave], the MapPoint's world position. A slot's MapPoint is the local-map search's match when it
// made one (SearchByProjection(F, vpMapPoints) overwrites a slot whose MapPoint has no observations), else the motion
// search's (an index into the last frame's entries). edge_kp[e] = i.
struct FrameEdgeArgs {
    const mam_keypoint* kps;
    int kp_stride;
    const int32_t* kp_count;
    int count_stride;
    float inv_sigma2[MAM_MAX_LEVELS];
    int nlevels;
    const int32_t* match_last;
    const mam_last_entry* last;
    int last_stride;
    const int32_t* match_local;
    const mam_local_mp* local;
    int local_stride;
    mam_pose_edge* edges;
    int edge_stride;
    int32_t* n_edges;
    int32_t* edge_kp;
};

// grid (nframes) x 256: the slots in keypoint order, compacted by a block prefix count
__global__ __launch_bounds__(256) void k_frame_edges(FrameEdgeArgs a) {
    __shared__ int wsum[4];
    __shared__ int base_s;
    const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int n = min(max(a.kp_count[(size_t)f * a.count_stride], 0), a.kp_stride);
    const mam_keypoint* K = a.kps + (size_t)f * a.kp_stride;
    const int32_t* ml = a.match_last + (size_t)f * a.kp_stride;
    const int32_t* mo = a.match_local ? a.match_local + (size_t)f * a.kp_stride : nullptr;
    mam_pose_edge* E = a.edges + (size_t)f * a.edge_stride;
    int32_t* EK = a.edge_kp + (size_t)f * a.edge_stride;
    if (t == 0) base_s = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += 256) {
        const int i = c0 + t;
        int jl = -1, jm = -1;
        if (i < n) {
            jm = mo ? mo[i] : -1;
            jl = ml[i];
        }
        const bool has = jm >= 0 || jl >= 0;
        const uint64_t m = __ballot(has);
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int off = base_s;
        for (int k = 0; k < w; k++) off += wsum[k];
        const int r = off + __popcll(m & ((1ull << lane) - 1ull));
        if (has && r < a.edge_stride) {
            const mam_keypoint kp = K[i];
            mam_pose_edge e;
            e.obs[0] = kp.x;
            e.obs[1] = kp.y;
            const float* X = jm >= 0 ? a.local[(size_t)f * a.local_stride + jm].pos
                                     : a.last[(size_t)f * a.last_stride + jl].pos;
            e.xw[0] = X[0];
            e.xw[1] = X[1];
            e.xw[2] = X[2];
            e.inv_sigma2 = a.inv_sigma2[min(max(kp.octave, 0), a.nlevels - 1)];
            E[r] = e;
            EK[r] = i;
        }
        __syncthreads();
        if (t == 0) base_s += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
    if (t == 0) a.n_edges[f] = base_s <= a.edge_stride ? base_s : MAM_ERR_CAPACITY;
}

// grid (ceil(nframes * edge_stride / 256)): Tracking's use of the result — Frame::SetPose(SE3f(q.cast<float>(),
// t.cast<float>())) (Sophus normalises the float quaternion; Optimizer.cc:1108-1111) and, with discard, the outliers'
// slots emptied (Tracking.cc:2840-2857: mvpMapPoints[i] = NULL — no match, not taken by the local-map search)
__global__ __launch_bounds__(256) void k_frame_update(int nframes, const mam_pose_result* __restrict__ res,
                                                      mam_pose* __restrict__ tcw, const uint8_t* __restrict__ outlier,
                                                      const int32_t* __restrict__ edge_kp, int edge_stride,
                                                      const int32_t* __restrict__ n_edges, int discard,
                                                      int32_t* __restrict__ match_last, uint8_t* __restrict__ taken,
                                                      int kp_stride) {
    const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
    const int f = (int)(g / (size_t)max(edge_stride, 1)), e = (int)(g % (size_t)max(edge_stride, 1));
    if (f >= nframes) return;
    const mam_pose_result& R = res[f];
    if (e == 0 && R.n_inliers >= 0 && R.rounds > 0) {
        float q[4];
        for (int k = 0; k < 4; k++) q[k] = (float)R.q[k];
        // Sophus SO3::normalize: coeffs / norm(), Eigen's SSE 4-float reduction (x^2 + z^2) + (y^2 + w^2)
        const float nq = sqrtf((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]));
        for (int k = 0; k < 4; k++) tcw[f].q[k] = q[k] / nq;
        for (int k = 0; k < 3; k++) tcw[f].t[k] = (float)R.t[k];
    }
    if (!discard || e >= n_edges[f] || !outlier[(size_t)f * edge_stride + e]) return;
    const int i = edge_kp[(size_t)f * edge_stride + e];
    match_last[(size_t)f * kp_stride + i] = -1;
    if (taken) taken[(size_t)f * kp_stride + i] = 0;
}

}  // namespace pose
}  // namespace mam

// ==================================================================================================== host
struct mam_pose_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int cap = 0;
    size_t lds = 0;
    mam::StageTimer timer{1};
    mam::DevBuf<uint8_t> stage;
};

extern "C" {

int mam_pose_create(int device, mam_pose_ctx** out) {
    if (!out) return MAM_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    MAM_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) { mam::set_last_error("no such HIP device"); return MAM_ERR_ARG; }
    MAM_DEVICE_SCOPE(device);
    mam_pose_ctx* c = new mam_pose_ctx();
    c->device = device;
    // LDS carve: as many edges as fit in 160 KB next to the kernel's static scratch
    size_t lim = 64 * 1024;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::pose::k_pose_opt<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::pose::k_pose_opt<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess)
        lim = 150 * 1024;
    else
        (void)hipGetLastError();
    int cap = 64;
    while (mam::pose::lds_bytes(cap + 64) <= lim) cap += 64;
    c->cap = cap;
    c->lds = mam::pose::lds_bytes(cap);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        mam::set_last_error("hipStreamCreate failed");
        return MAM_ERR_DEVICE;
    }
    *out = c;
    return MAM_OK;
}

void mam_pose_destroy(mam_pose_ctx* c) {
    if (!c) return;
    ::mam::DeviceScope mam_dev_scope_(c->device);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int mam_pose_max_edges(mam_pose_ctx* c) { return c ? c->cap : MAM_ERR_ARG; }

int mam_pose_optimization_batch_device(mam_pose_ctx* c, int nframes, const mam_pose* tcw, const mam_camera* cam,
                                       const mam_pose_edge* edges, int edge_stride, const int32_t* n_edges,
                                       uint8_t* outlier, mam_pose_result* results, void* stream) {
    if (!c || nframes < 0 || !cam || edge_stride < 0) return MAM_ERR_ARG;
    if (nframes == 0) return MAM_OK;
    if (!tcw || !n_edges || !results || (edge_stride > 0 && (!edges || !outlier))) return MAM_ERR_ARG;
    if (edge_stride > c->cap) {
        mam::set_last_error("edge_stride exceeds mam_pose_max_edges()");
        return MAM_ERR_CAPACITY;
    }
    MAM_DEVICE_SCOPE(c->device);
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    mam::pose::Args a;
    a.nframes = nframes;
    a.tcw = tcw;
    a.cam = *cam;
    a.edges = edges;
    a.stride = edge_stride;
    a.n_edges = n_edges;
    a.outlier = outlier;
    a.res = results;
    // the LDS carve sized to the edge stride (a frame's edges never exceed it), not to the context's capacity: a c2
    // frame's 2k-edge stride takes ~82 KB instead of 150, and the rest of the CU's LDS stays free for the other
    // lanes' kernels (extraction, matching) running beside the optimisation
    a.cap = std::min(c->cap, std::max(64, (edge_stride + 63) / 64 * 64));
    const size_t lds = mam::pose::lds_bytes(a.cap);
    {
        mam::StageTimer::Scope sc(&c->timer, s, 0);
        if (cam->model == MAM_CAM_KANNALA_BRANDT8)
            hipLaunchKernelGGL(mam::pose::k_pose_opt<true>, dim3(nframes), dim3(mam::pose::Cfg<true>::PT), lds, s, a);
        else
            hipLaunchKernelGGL(mam::pose::k_pose_opt<false>, dim3(nframes), dim3(mam::pose::Cfg<false>::PT), lds, s, a);
    }
    MAM_HIP(hipGetLastError());
#ifdef MAM_POSE_PROFILE
    {
        MAM_HIP(hipStreamSynchronize(s));
        unsigned long long h[16];
        MAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(mam::pose::g_pprof), sizeof(h)));
        fprintf(stderr, "pose reduce: scatter %.0f barrier1 %.0f sum+barrier2 %.0f /pass; ldlt6 %.0f exp %.0f /trial\n",
                h[8] / (double)std::max(1ull, h[6]), h[9] / (double)std::max(1ull, h[6]),
                h[10] / (double)std::max(1ull, h[6]), h[11] / (double)std::max(1ull, h[5]),
                h[12] / (double)std::max(1ull, h[5]));
        const double nb = (double)std::max(1ull, h[6]), nt = (double)std::max(1ull, h[5]);
        fprintf(stderr, "pose cycles (cumulative): build %.0f/pass (edge loop %.0f) ldlt %.0f exp %.0f trial %.0f/trial "
                        "control %.0f; builds %llu trials %llu\n", h[0] / nb, h[7] / nb, h[1] / nt, h[2] / nt, h[3] / nt,
                h[4] / nt, h[6], h[5]);
    }
#endif
    return MAM_OK;
}

int mam_pose_optimization(mam_pose_ctx* c, const mam_pose* tcw, const mam_camera* cam, int n,
                          const mam_pose_edge* edges, uint8_t* outlier, mam_pose_result* result) {
    if (!c || !tcw || !cam || n < 0 || (n > 0 && (!edges || !outlier)) || !result) return MAM_ERR_ARG;
    if (n > c->cap) {
        mam::set_last_error("more edges than mam_pose_max_edges()");
        return MAM_ERR_CAPACITY;
    }
    MAM_DEVICE_SCOPE(c->device);
    const size_t S = std::max(n, 1);
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bytes = al(S * sizeof(mam_pose_edge)) + al(S) + al(sizeof(mam_pose_result)) + al(sizeof(mam_pose)) + al(4);
    if (int rc = c->stage.alloc(bytes)) return rc;
    uint8_t* p = c->stage.p;
    mam_pose_edge* de = reinterpret_cast<mam_pose_edge*>(p); p += al(S * sizeof(mam_pose_edge));
    uint8_t* dout = p;                                       p += al(S);
    mam_pose_result* dres = reinterpret_cast<mam_pose_result*>(p); p += al(sizeof(mam_pose_result));
    mam_pose* dp = reinterpret_cast<mam_pose*>(p);           p += al(sizeof(mam_pose));
    int32_t* dn = reinterpret_cast<int32_t*>(p);
    if (n > 0) MAM_HIP(hipMemcpyAsync(de, edges, sizeof(mam_pose_edge) * n, hipMemcpyHostToDevice, c->stream));
    MAM_HIP(hipMemcpyAsync(dp, tcw, sizeof(mam_pose), hipMemcpyHostToDevice, c->stream));
    MAM_HIP(hipMemcpyAsync(dn, &n, 4, hipMemcpyHostToDevice, c->stream));
    if (int rc = mam_pose_optimization_batch_device(c, 1, dp, cam, de, (int)S, dn, dout, dres, c->stream)) return rc;
    if (n > 0) MAM_HIP(hipMemcpyAsync(outlier, dout, n, hipMemcpyDeviceToHost, c->stream));
    MAM_HIP(hipMemcpyAsync(result, dres, sizeof(mam_pose_result), hipMemcpyDeviceToHost, c->stream));
    MAM_HIP(hipStreamSynchronize(c->stream));
    return result->n_inliers;
}

int mam_pose_frame_edges_batch_device(mam_pose_ctx* c, int nframes, const mam_keypoint* kps, int kp_stride,
                                      const int32_t* kp_count, int count_stride, const float* inv_level_sigma2,
                                      int nlevels, const int32_t* match_last, const mam_last_entry* last,
                                      int last_stride, const int32_t* match_local, const mam_local_mp* local_mps,
                                      int local_stride, mam_pose_edge* edges, int edge_stride, int32_t* n_edges,
                                      int32_t* edge_kp, void* stream) {
    if (!c || nframes < 0 || kp_stride < 0 || count_stride < 1 || nlevels < 1 || nlevels > MAM_MAX_LEVELS ||
        !inv_level_sigma2 || edge_stride < 0)
        return MAM_ERR_ARG;
    if (nframes == 0) return MAM_OK;
    if (!kps || !kp_count || !match_last || !last || !edges || !n_edges || !edge_kp ||
        (match_local && !local_mps))
        return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    mam::pose::FrameEdgeArgs a{};
    a.kps = kps;
    a.kp_stride = kp_stride;
    a.kp_count = kp_count;
    a.count_stride = count_stride;
    for (int l = 0; l < nlevels; l++) a.inv_sigma2[l] = inv_level_sigma2[l];
    a.nlevels = nlevels;
    a.match_last = match_last;
    a.last = last;
    a.last_stride = last_stride;
    a.match_local = match_local;
    a.local = local_mps;
    a.local_stride = local_stride;
    a.edges = edges;
    a.edge_stride = edge_stride;
    a.n_edges = n_edges;
    a.edge_kp = edge_kp;
    hipLaunchKernelGGL(mam::pose::k_frame_edges, dim3(nframes), dim3(256), 0, s, a);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

int mam_pose_frame_update_batch_device(mam_pose_ctx* c, int nframes, const mam_pose_result* results, mam_pose* tcw,
                                       const uint8_t* outlier, const int32_t* edge_kp, int edge_stride,
                                       const int32_t* n_edges, int discard, int32_t* match_last, uint8_t* taken,
                                       int kp_stride, void* stream) {
    if (!c || nframes < 0 || edge_stride < 0 || kp_stride < 0) return MAM_ERR_ARG;
    if (nframes == 0) return MAM_OK;
    if (!results || !tcw || !n_edges || (discard && (!outlier || !edge_kp || !match_last))) return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    const size_t total = (size_t)nframes * (size_t)std::max(edge_stride, 1);
    hipLaunchKernelGGL(mam::pose::k_frame_update, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, nframes,
                       results, tcw, outlier, edge_kp, edge_stride, n_edges, discard, match_last, taken, kp_stride);
    MAM_HIP(hipGetLastError());
    return MAM_OK;
}

int mam_pose_set_profiling(mam_pose_ctx* c, int enable) {
    if (!c) return MAM_ERR_ARG;
    c->timer.collect();
    c->timer.reset(enable != 0);
    return MAM_OK;
}

int mam_pose_stage_times(mam_pose_ctx* c, double* ms_out, int64_t* launches_out) {
    if (!c || !ms_out || !launches_out) return MAM_ERR_ARG;
    c->timer.collect();
    ms_out[0] = c->timer.ms[0];
    launches_out[0] = c->timer.n[0];
    return MAM_OK;
}

}  // extern "C"
