// lba.hip — gfx950 Levenberg-Marquardt / Schur solve of Optimizer::LocalBundleAdjustment (include/mam_lba.h).
//
// g2o semantics (BlockSolver_6_3 + LinearSolverEigen + OptimizationAlgorithmLevenberg, FP64) re-laid out for
// the GPU; every reduction has a fixed order so results are run-to-run reproducible:
//   k_linearize   per edge: map, error, chi2, Huber rho, Jacobians (OptimizableTypes.cpp:139-160), the
//                 robust-weighted terms constructQuadraticForm needs (base_binary_edge.hpp:75-112)
//   k_point_sys   per point: H_ll, b_l over its edge segment (insertion order) and per-edge H_pl = B^T W A
//   k_pose_sys    one wave per non-fixed pose: lanes own the 36+6 entries of H_pp, b_p; edges in order
//   k_schur_prep  per point: D = H_ll + lambda I, D^-1, D^-1 b_l, per-edge H_pl D^-1 and H_pl D^-1 b_l
//   k_schur_blk   one wave per 6x6 block (i1 <= i2) of the reduced camera system: lanes own entries,
//                 contributions summed in landmark order (block_solver.hpp:372-439)
//   k_schur_rhs   b_s = b_p - sum coefficients
//   k_ldlt        single-workgroup blocked right-looking LDL^T of S (zero pivot = failure, as SimplicialLDLT)
//                 + forward / diagonal / backward substitution
//   k_backsub     x_l = D^-1 (b_l - H_pl^T x_p)  (block_solver.hpp:461-482)
//   k_update      T <- exp(dx) T (se3quat.h), X <- X + dx on the trial copy
//   k_chi2        robust chi2 of the trial state + computeScale terms; fixed-order block reduction
// The LM control flow (levenberg.cpp:61-169) stays on the host and reads 3 scalars per trial.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <limits>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/mam_lba.h"
#include "runtime.hpp"

namespace mam {
namespace lba {

struct Dev {
    // problem
    int P, L, E, Np;
    const int32_t* edge_point;
    const int32_t* edge_pose;
    const double* edge_obs;
    const double* edge_w;        // invSigma2
    const float* cams;
    const int32_t* pose_cam;
    const int32_t* pose_h;       // Hessian pose block of pose (-1 fixed)
    const int32_t* hpose;        // Hessian pose block -> pose
    const int32_t* point_h;      // Hessian point of point
    const int32_t* hpoint;       // Hessian point -> point
    const int32_t* pe_off;       // per Hessian point: edge segment [pe_off[h], pe_off[h+1]) into pe_idx
    const int32_t* pe_idx;
    const int32_t* qe_off;       // per Hessian pose: edges
    const int32_t* qe_idx;
    const int32_t* bp_ij;        // (i1 <= i2) per block of the upper triangle of S, row-major
    int nbp;
    int32_t* eidx;               // [Np][L] edge of (pose block, Hessian point), -1 if none
    int npad;                    // padded dimension of S (ldlt_pad(6 Np))
    double* ws;                  // global LDL^T workspace when it does not fit in LDS
    double delta;                // Huber delta; <= 0: no robust kernel
    const uint8_t* active;       // [E] level-0 edges (NULL = all)
    // state
    const double* pose;          // [P][7] q(xyzw) t
    const double* pt;            // [L][3]
    double* pose_out;            // trial
    double* pt_out;
    // per edge
    double* err;                 // [E][2]
    double* jac;                 // [E][21]: A(6) B(12) orr(2) wo(1)
    double* rho0;                // [E]
    double* part;                // [ceil(E / 256)] rho0 partial sums of k_linearize's blocks
    double* hpl;                 // [E][18] H_pl pose x landmark
    double* bdinv;               // [E][18] H_pl D^-1
    double* coef;                // [E][6]  H_pl D^-1 b_l
    // system
    double* Hpp;                 // [Np][36]
    double* Hll;                 // [L][9] (Hessian point order)
    double* b;                   // [6Np + 3L]
    double* Dinv;                // [L][9]
    double* S;                   // [n][n]
    double* x;                   // [6Np + 3L]
    double* bs;                  // [6Np]
    double* red;                 // reduction scratch
    int* flag;
};

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

__device__ __forceinline__ void huber(double e, double delta, double* r0, double* r1) {
    const double dsqr = delta * delta;
    if (delta <= 0.0 || e <= dsqr) { *r0 = e; *r1 = 1.0; }   // no kernel: rho(e) = e, rho' = 1
    else {
        const double s = sqrt(e);
        *r0 = 2 * s * delta - dsqr;
        *r1 = delta / s;
    }
}

// ---- per edge: error, robust weight, Jacobians (EdgeSE3ProjectXYZ); returns the edge's rho0
__device__ __forceinline__ double linearize_edge(const Dev& d, int e, int want_jac) {
    const int ip = d.edge_point[e] , ipose = d.edge_pose[e];
    const double* T = d.pose + 7 * (size_t)ipose;
    const double* X = d.pt + 3 * (size_t)ip;
    double Xc[3];
    map_point(T, X, Xc);
    const float* c = d.cams + 4 * (d.pose_cam ? d.pose_cam[ipose] : 0);
    const double fx = c[0], fy = c[1];
    const double u = c[0] * Xc[0] / Xc[2] + c[2];
    const double v = c[1] * Xc[1] / Xc[2] + c[3];
    const double e0 = d.edge_obs[2 * e] - u, e1 = d.edge_obs[2 * e + 1] - v;
    d.err[2 * e] = e0;
    d.err[2 * e + 1] = e1;
    if (d.active && !d.active[e]) {
        // setLevel(1): outside initializeOptimization(0), no term in chi2 / H / b (zeros add exactly nothing)
        d.rho0[e] = 0.0;
        if (want_jac) {
            double* o = d.jac + 21 * (size_t)e;
            for (int k = 0; k < 21; k++) o[k] = 0.0;
            if (d.pose_h[ipose] >= 0)
                for (int k = 0; k < 18; k++) d.hpl[18 * (size_t)e + k] = 0.0;
        }
        return 0.0;
    }
    const double w = d.edge_w[e];
    const double chi = e0 * (w * e0) + e1 * (w * e1);
    double r0, r1;
    huber(chi, d.delta, &r0, &r1);
    d.rho0[e] = r0;
    if (!want_jac) return r0;
    const double x = Xc[0], y = Xc[1], z = Xc[2];
    const double J0 = -(fx / z), J2 = -(-fx * x / (z * z)), J4 = -(fy / z), J5 = -(-fy * y / (z * z));
    // rotation matrix of T (Eigen toRotationMatrix)
    const double qx = T[0], qy = T[1], qz = T[2], qw = T[3];
    const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
    const double twx = tx * qw, twy = ty * qw, twz = tz * qw, txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                         txz - twy, tyz + twx, 1 - (txx + tyy)};
    double* o = d.jac + 21 * (size_t)e;
    // A = J R (2x3), J = [[J0, 0, J2], [0, J4, J5]]
    for (int k = 0; k < 3; k++) {
        o[k] = J0 * R[k] + J2 * R[6 + k];
        o[3 + k] = J4 * R[3 + k] + J5 * R[6 + k];
    }
    // B = J * SE3deriv, SE3deriv = [[0,z,-y,1,0,0],[-z,0,x,0,1,0],[y,-x,0,0,0,1]]
    o[6] = J2 * y;  o[7] = J0 * z - J2 * x; o[8] = -J0 * y; o[9] = J0; o[10] = 0.0; o[11] = J2;
    o[12] = -J4 * z + J5 * y; o[13] = -J5 * x; o[14] = J4 * x; o[15] = 0.0; o[16] = J4; o[17] = J5;
    o[18] = -(w * e0) * r1;
    o[19] = -(w * e1) * r1;
    o[20] = r1 * w;
    // H_pl = B^T (rho' Omega) A for edges whose pose is optimised (base_binary_edge.hpp:54-120)
    if (d.pose_h[ipose] >= 0) {
        const double wo = r1 * w;
        double* hp = d.hpl + 18 * (size_t)e;
        for (int a = 0; a < 6; a++)
            for (int c = 0; c < 3; c++) hp[3 * a + c] = o[6 + a] * wo * o[c] + o[12 + a] * wo * o[3 + c];
    }
    return r0;
}

// Per block of 256 edges: the rho0 partial sum in a fixed order (butterfly per wave, then the 4 waves in order), so
// the chi2 reduction is one short pass over the partials
__global__ __launch_bounds__(256) void k_linearize(Dev d, int want_jac) {
    __shared__ double ws[4];
    const int e = blockIdx.x * 256 + threadIdx.x;
    double r = e < d.E ? linearize_edge(d, e, want_jac) : 0.0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = r;
    __syncthreads();
    if (threadIdx.x == 0) d.part[blockIdx.x] = ((ws[0] + ws[1]) + ws[2]) + ws[3];
}

// ---- per point: H_ll, b_l (edge order, as constructQuadraticForm runs edge by edge)
__global__ __launch_bounds__(64) void k_point_sys(Dev d) {
    const int h = blockIdx.x * 64 + threadIdx.x;
    if (h >= d.L) return;
    double H[9] = {0}, bl[3] = {0};
    for (int s = d.pe_off[h]; s < d.pe_off[h + 1]; s++) {
        const int e = d.pe_idx[s];
        const double* j = d.jac + 21 * (size_t)e;
        const double wo = j[20];
        for (int a = 0; a < 3; a++) {
            bl[a] += j[a] * j[18] + j[3 + a] * j[19];
            for (int c = 0; c < 3; c++) H[3 * a + c] += j[a] * wo * j[c] + j[3 + a] * wo * j[3 + c];
        }
    }
    for (int k = 0; k < 9; k++) d.Hll[9 * (size_t)h + k] = H[k];
    for (int k = 0; k < 3; k++) d.b[6 * (size_t)d.Np + 3 * (size_t)h + k] = bl[k];
}

// fixed-order (butterfly) wave sum: every lane ends with the same value, deterministic run to run
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---- one wave per non-fixed pose: lanes stride over the pose's edges, accumulate the 21 upper entries of
// H_pp and the 6 of b_p in registers, then a fixed-order wave reduction
__global__ __launch_bounds__(64) void k_pose_sys(Dev d) {
    const int h = blockIdx.x, lane = threadIdx.x;
    double acc[27];
#pragma unroll
    for (int k = 0; k < 27; k++) acc[k] = 0.0;
    for (int s = d.qe_off[h] + lane; s < d.qe_off[h + 1]; s += 64) {
        const double* j = d.jac + 21 * (size_t)d.qe_idx[s];
        double B0[6], B1[6];
#pragma unroll
        for (int k = 0; k < 6; k++) { B0[k] = j[6 + k]; B1[k] = j[12 + k]; }
        const double wo = j[20], o0 = j[18], o1 = j[19];
        int q = 0;
#pragma unroll
        for (int a = 0; a < 6; a++)
#pragma unroll
            for (int c = a; c < 6; c++) acc[q++] += B0[a] * wo * B0[c] + B1[a] * wo * B1[c];
#pragma unroll
        for (int a = 0; a < 6; a++) acc[21 + a] += B0[a] * o0 + B1[a] * o1;
    }
#pragma unroll
    for (int k = 0; k < 27; k++) acc[k] = wave_sum_d(acc[k]);
    if (lane == 0) {
        int q = 0;
        double* H = d.Hpp + 36 * (size_t)h;
        for (int a = 0; a < 6; a++)
            for (int c = a; c < 6; c++) { H[6 * a + c] = acc[q]; H[6 * c + a] = acc[q]; q++; }
        for (int a = 0; a < 6; a++) d.b[6 * (size_t)h + a] = acc[21 + a];
    }
}

// ---- fixed-order sum of rho0 (and max diag) in one workgroup. RED threads: a small workgroup finds room on a CU
// that Tracking's concurrent launches keep busy (a 1024-thread one waits for 16 free wave slots at once).
#ifndef MAM_LBA_RED_THREADS
#define MAM_LBA_RED_THREADS 256
#endif
constexpr int RED = MAM_LBA_RED_THREADS;

__global__ __launch_bounds__(RED) void k_reduce_chi(Dev d, int slot) {
    __shared__ double s[RED];
    const int t = threadIdx.x;
    double acc = 0.0;
    const int nb = (d.E + 255) / 256;
    for (int b = t; b < nb; b += RED) acc += d.part[b];
    s[t] = acc;
    __syncthreads();
    for (int o = RED / 2; o > 0; o >>= 1) {
        if (t < o) s[t] += s[t + o];
        __syncthreads();
    }
    if (t == 0) d.red[slot] = s[0];
}

__global__ __launch_bounds__(RED) void k_max_diag(Dev d) {
    __shared__ double s[RED];
    const int t = threadIdx.x;
    double m = 0.0;
    for (int i = t; i < 6 * d.Np; i += RED) m = fmax(m, fabs(d.Hpp[36 * (size_t)(i / 6) + 7 * (i % 6)]));
    for (int i = t; i < 3 * d.L; i += RED) m = fmax(m, fabs(d.Hll[9 * (size_t)(i / 3) + 4 * (i % 3)]));
    s[t] = m;
    __syncthreads();
    for (int o = RED / 2; o > 0; o >>= 1) {
        if (t < o) s[t] = fmax(s[t], s[t + o]);
        __syncthreads();
    }
    if (t == 0) d.red[2] = s[0];
}

// ---- Schur
__global__ __launch_bounds__(64) void k_schur_prep(Dev d, double lambda) {
    const int h = blockIdx.x * 64 + threadIdx.x;
    if (h >= d.L) return;
    double D[9];
    for (int k = 0; k < 9; k++) D[k] = d.Hll[9 * (size_t)h + k] + ((k % 4 == 0) ? lambda : 0.0);
    const double c00 = D[4] * D[8] - D[5] * D[7], c01 = D[5] * D[6] - D[3] * D[8], c02 = D[3] * D[7] - D[4] * D[6];
    const double det = D[0] * c00 + D[1] * c01 + D[2] * c02;
    double Di[9];
    Di[0] = c00 / det; Di[3] = c01 / det; Di[6] = c02 / det;
    Di[1] = (D[2] * D[7] - D[1] * D[8]) / det; Di[4] = (D[0] * D[8] - D[2] * D[6]) / det;
    Di[7] = (D[1] * D[6] - D[0] * D[7]) / det;
    Di[2] = (D[1] * D[5] - D[2] * D[4]) / det; Di[5] = (D[2] * D[3] - D[0] * D[5]) / det;
    Di[8] = (D[0] * D[4] - D[1] * D[3]) / det;
    for (int k = 0; k < 9; k++) d.Dinv[9 * (size_t)h + k] = Di[k];
}

// per edge (optimised pose): H_pl D^-1 and the coefficient H_pl D^-1 b_l (block_solver.hpp:405-427)
__global__ __launch_bounds__(256) void k_schur_edge(Dev d) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= d.E || d.pose_h[d.edge_pose[e]] < 0) return;
    const int h = d.point_h[d.edge_point[e]];
    const double* Di = d.Dinv + 9 * (size_t)h;
    const double* bl = d.b + 6 * (size_t)d.Np + 3 * (size_t)h;
    double db[3];
    for (int i = 0; i < 3; i++) db[i] = Di[3 * i] * bl[0] + Di[3 * i + 1] * bl[1] + Di[3 * i + 2] * bl[2];
    const double* B = d.hpl + 18 * (size_t)e;
    double* o = d.bdinv + 18 * (size_t)e;
    double* cf = d.coef + 6 * (size_t)e;
    for (int i = 0; i < 6; i++) {
        for (int j = 0; j < 3; j++) o[3 * i + j] = B[3 * i] * Di[j] + B[3 * i + 1] * Di[3 + j] + B[3 * i + 2] * Di[6 + j];
        cf[i] = B[3 * i] * db[0] + B[3 * i + 1] * db[1] + B[3 * i + 2] * db[2];
    }
}

__global__ __launch_bounds__(256) void k_eidx(Dev d) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= d.E) return;
    const int hp = d.pose_h[d.edge_pose[e]];
    if (hp >= 0) d.eidx[(size_t)hp * d.L + d.point_h[d.edge_point[e]]] = e;
}

__global__ __launch_bounds__(64) void k_schur_blk(Dev d, double lambda) {
    const int bp = blockIdx.x, lane = threadIdx.x;
    const int i1 = d.bp_ij[2 * bp], i2 = d.bp_ij[2 * bp + 1];
    double acc[36];
#pragma unroll
    for (int k = 0; k < 36; k++) acc[k] = 0.0;
    // landmarks seen by both poses: walk pose i2's edges, look up pose i1's edge of the same landmark
    const int32_t* ei1 = d.eidx + (size_t)i1 * d.L;
    for (int s = d.qe_off[i2] + lane; s < d.qe_off[i2 + 1]; s += 64) {
        const int ec = d.qe_idx[s];
        const int ea = ei1[d.point_h[d.edge_point[ec]]];
        if (ea < 0) continue;
        const double* W = d.bdinv + 18 * (size_t)ea;
        const double* B = d.hpl + 18 * (size_t)ec;
        double w[18], b[18];
#pragma unroll
        for (int k = 0; k < 18; k++) { w[k] = W[k]; b[k] = B[k]; }
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = 0; c < 6; c++) acc[6 * r + c] += w[3 * r] * b[3 * c] + w[3 * r + 1] * b[3 * c + 1] + w[3 * r + 2] * b[3 * c + 2];
    }
#pragma unroll
    for (int k = 0; k < 36; k++) acc[k] = wave_sum_d(acc[k]);
    if (lane < 36) {
        const int r = lane / 6, c = lane % 6;
        double v = 0.0;
#pragma unroll
        for (int k = 0; k < 36; k++) v = (k == lane) ? acc[k] : v;
        double out = -v;
        if (i1 == i2) out = (d.Hpp[36 * (size_t)i1 + lane] + (r == c ? lambda : 0.0)) - v;
        const int N = d.npad;
        d.S[(size_t)(6 * i1 + r) * N + 6 * i2 + c] = out;
        d.S[(size_t)(6 * i2 + c) * N + 6 * i1 + r] = out;
    }
}

// b_s = b_p - sum of the pose's coefficients: lanes stride the pose's edges, fixed-order wave reduction
__global__ __launch_bounds__(64) void k_schur_rhs(Dev d) {
    const int h = blockIdx.x, lane = threadIdx.x;
    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int s = d.qe_off[h] + lane; s < d.qe_off[h + 1]; s += 64) {
        const double* c = d.coef + 6 * (size_t)d.qe_idx[s];
#pragma unroll
        for (int k = 0; k < 6; k++) acc[k] += c[k];
    }
#pragma unroll
    for (int k = 0; k < 6; k++) acc[k] = wave_sum_d(acc[k]);
    if (lane < 6) {
        double v = 0.0;
#pragma unroll
        for (int k = 0; k < 6; k++) v = (k == lane) ? acc[k] : v;
        d.bs[6 * (size_t)h + lane] = d.b[6 * (size_t)h + lane] - v;
    }
}

// ---- dense LDL^T solve of S x = bs: one workgroup of 1024 threads, blocked right-looking, NB = 16 panels.
// S is npad x npad (npad = 6 Np rounded up to 16; the padding is an identity block after the real unknowns, so it
// changes nothing and every panel is full). Per panel:
//   (1) wave 0 factors the 16x16 diagonal block in registers: lane i owns row i, the pivot row is read with
//       v_readlane (uniform), and solves the block of the forward substitution L11 y1 = y1;
//   (2) every thread takes one panel row: L21 = A21 L11^-T D^-1, W21 = L21 D (staged transposed in the panel
//       workspace for the trailing update) and the fused forward-substitution update y2 -= L21 y1;
//   (3) the trailing lower triangle A22 -= L21 W21^T in 16x16 blocks, one wave each, as f64 MFMAs
//       (v_mfma_f64_16x16x4_f64) with both operands from the workspace.
// An exact zero pivot sets flag[0] (the failure rule of Eigen's SimplicialLDLT) and skips the solve.
// Then y /= D and the backward substitution L^T x = y, block by block, each thread updating its own y_i.
// The workspace (panel + y) is LDS when it fits (use_lds), else a global scratch buffer.
constexpr int NB = 16;
#ifndef MAM_LDLT_THREADS
#define MAM_LDLT_THREADS 512
#endif
constexpr int LDLT_THREADS = MAM_LDLT_THREADS;   // 16 waves: 4 per SIMD hide the MFMA / memory latency

__host__ __device__ inline int ldlt_pad(int n) { return (n + NB - 1) / NB * NB; }

// workspace doubles: PL and PW (NB x (npad - NB) each) + y (npad)
__host__ __device__ inline size_t ldlt_ws_doubles(int npad) {
    const int m = npad > NB ? npad - NB : 0;
    return (size_t)2 * NB * (size_t)m + (size_t)npad;
}
__host__ __device__ inline size_t ldlt_lds_bytes(int npad) { return ldlt_ws_doubles(npad) * sizeof(double); }

__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), l);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// wave 0: LDL^T of the 16x16 diagonal block at kb (final on entry), written back to A (L below, D on the diagonal),
// plus Ld (L11, row-major), dk / invdk (D and 1/D) for the panel rows, and the forward block solve of y.
// Right-looking inside the block: at step j the pivot d_j is lane j's current diagonal, column j is scaled
// (l_ij = a_ij / d_j) and broadcast by v_readlane, and every lane i > j updates a_ik -= l_ij d_j l_kj, j < k <= i.
__device__ __forceinline__ void ldlt_diag(double* A, int N, int kb, double* Y, double* Ld, double* dk, double* invdk,
                                          int* fail, int lane) {
    double row[NB];
#pragma unroll
    for (int c = 0; c < NB; c++) row[c] = lane < NB ? A[(size_t)(kb + lane) * N + kb + c] : 0.0;
    double dmine = 1.0;
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const double dj = readlane_d(row[j], j);
        if (lane == j) dmine = dj;
        const double inv = dj != 0.0 ? 1.0 / dj : 0.0;
        const double l = row[j] * inv;
        if (lane > j) row[j] = l;
        const double ldj = l * dj;
#pragma unroll
        for (int k = j + 1; k < NB; k++) {
            const double lk = readlane_d(l, k);
            if (k <= lane) row[k] -= ldj * lk;
        }
    }
    double yv = lane < NB ? Y[kb + lane] : 0.0;
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const double yj = readlane_d(yv, j);
        if (lane > j) yv -= row[j] * yj;
    }
    if (lane < NB) {
#pragma unroll
        for (int c = 0; c < NB; c++) {
            Ld[lane * NB + c] = row[c];
            if (c < lane) A[(size_t)(kb + lane) * N + kb + c] = row[c];
        }
        A[(size_t)(kb + lane) * N + kb + lane] = dmine;
        dk[lane] = dmine;
        invdk[lane] = dmine != 0.0 ? 1.0 / dmine : 0.0;
        Y[kb + lane] = yv;
        if (dmine == 0.0) *fail = 1;
    }
}

// One wave: the 16x16 block (br, bc) of A22 (block indices relative to row/col kb + NB) -= L21 W21^T as four
// chained v_mfma_f64_16x16x4_f64 (K = 16), accumulator initialised with the A block. Lane maps (gfx950, f64):
// A operand L[R0 + (lane&15)][k0 + (lane>>4)], B operand W[C0 + (lane&15)][k0 + (lane>>4)],
// C/D col = lane&15, row = (lane>>4) + 4 reg.
typedef double dbl4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ldlt_tile16(double* A, int N, int kb, const double* PL, const double* PW, int m, int br,
                                            int bc, int lane) {
    const int R0 = kb + NB + 16 * br, C0 = kb + NB + 16 * bc;
    const int col = lane & 15, rq = lane >> 4;
    dbl4 c;
#pragma unroll
    for (int r = 0; r < 4; r++) c[r] = A[(size_t)(R0 + rq + 4 * r) * N + C0 + col];
#pragma unroll
    for (int k0 = 0; k0 < NB; k0 += 4) {
        const int k = k0 + rq;
        const double av = -PL[(size_t)k * m + 16 * br + col];
        const double bv = PW[(size_t)k * m + 16 * bc + col];
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) A[(size_t)(R0 + rq + 4 * r) * N + C0 + col] = c[r];
}

// triangle index q -> (tr, tc), tc <= tr
__device__ __forceinline__ void tri_index(int q, int* tr, int* tc) {
    int r = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
    while (r * (r + 1) / 2 > q) r--;
    while ((r + 1) * (r + 2) / 2 <= q) r++;
    *tr = r;
    *tc = q - r * (r + 1) / 2;
}

// With lookahead: after a panel's rows (B), the next block column is updated first (C1); then wave 0 factors the
// next diagonal block while the other waves update the rest of the trailing matrix (C2).
template <bool use_lds>
__global__ __launch_bounds__(LDLT_THREADS) void k_ldlt(Dev d) {
    extern __shared__ __attribute__((aligned(16))) double lds_ws[];
    const int n = 6 * d.Np, N = d.npad;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    double* A = d.S;
    double* ws = use_lds ? lds_ws : d.ws;
    double* Y = ws + (size_t)2 * NB * (N - NB);
    __shared__ double Ld[NB * NB];
    __shared__ double dk[NB];
    __shared__ double invdk[NB];
    __shared__ int fail;
    if (t == 0) fail = 0;
    for (int i = t; i < N; i += LDLT_THREADS) {
        Y[i] = d.bs[i];
        if (i >= n) A[(size_t)i * N + i] = 1.0;
    }
    __syncthreads();
#ifdef MAM_LDLT_PROFILE
    long long tp0 = clock64(), tacc[4] = {0, 0, 0, 0};
#define LDLT_PHASE(k) do { const long long tn = clock64(); tacc[k] += tn - tp0; tp0 = tn; } while (0)
#else
#define LDLT_PHASE(k) do {} while (0)
#endif
    if (wid == 0) ldlt_diag(A, N, 0, Y, Ld, dk, invdk, &fail, lane);
    __syncthreads();
    LDLT_PHASE(0);
    for (int kb = 0; kb < N; kb += NB) {
        // (B) panel rows: L21 = A21 L11^-T D^-1, W21 = L21 D (staged transposed), y2 -= L21 y1
        const int m = N - kb - NB;
        double* PL = ws;
        double* PW = ws + (size_t)NB * m;
        for (int i = kb + NB + t; i < N; i += LDLT_THREADS) {
            // keep the L11 factors in LDS (reading them per row): hoisting all 120 into registers spills
            asm volatile("" ::: "memory");
            double w[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) w[j] = A[(size_t)i * N + kb + j];
#pragma unroll
            for (int j = 1; j < NB; j++) {
#pragma unroll
                for (int k = 0; k < j; k++) w[j] -= w[k] * Ld[j * NB + k];
            }
            double yi = Y[i];
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const double lij = w[j] * invdk[j];
                A[(size_t)i * N + kb + j] = lij;
                PL[(size_t)j * m + (i - kb - NB)] = lij;
                PW[(size_t)j * m + (i - kb - NB)] = w[j];
                yi -= lij * Y[kb + j];
            }
            Y[i] = yi;
        }
        __syncthreads();
        LDLT_PHASE(1);
        if (m == 0) break;
        const int T16 = m / 16;
        // (C1) the next block column: blocks (br, 0), one wave each
        for (int br = wid; br < T16; br += LDLT_THREADS / 64) ldlt_tile16(A, N, kb, PL, PW, m, br, 0, lane);
        __syncthreads();
        LDLT_PHASE(2);
        // (C2) wave 0 factors the next diagonal block; the other waves update the blocks with bc >= 1
        if (wid == 0) {
            ldlt_diag(A, N, kb + NB, Y, Ld, dk, invdk, &fail, lane);
        } else {
            const int T2 = T16 - 1;
            const int n2 = T2 * (T2 + 1) / 2;
            for (int q = wid - 1; q < n2; q += LDLT_THREADS / 64 - 1) {
                int tr, tc;
                tri_index(q, &tr, &tc);
                ldlt_tile16(A, N, kb, PL, PW, m, tr + 1, tc + 1, lane);
            }
        }
        __syncthreads();
        LDLT_PHASE(0);
    }
#ifdef MAM_LDLT_PROFILE
    if (t == 0) for (int k = 0; k < 3; k++) d.red[4 + k] += (double)tacc[k];
#endif
    if (t == 0) d.flag[0] = fail;
    if (fail) return;   // uniform (LDS flag after the last barrier)
    // y /= D
    for (int i = t; i < N; i += LDLT_THREADS) Y[i] /= A[(size_t)i * N + i];
    __syncthreads();
    // backward substitution L^T x = y: block solve by wave 0, then each thread i < kb updates its own y_i
    for (int kb = N - NB; kb >= 0; kb -= NB) {
        if (wid == 0) {
            double col[NB];   // lane c holds L(kb + j, kb + c) for j > c
#pragma unroll
            for (int j = 0; j < NB; j++) col[j] = lane < NB ? A[(size_t)(kb + j) * N + kb + lane] : 0.0;
            double v = lane < NB ? Y[kb + lane] : 0.0;
#pragma unroll
            for (int j = NB - 1; j >= 0; j--) {
                const double xj = readlane_d(v, j);
                if (lane < j) v -= col[j] * xj;
            }
            if (lane < NB) Y[kb + lane] = v;
        }
        __syncthreads();
        for (int i = t; i < kb; i += LDLT_THREADS) {
            double sy = Y[i];
#pragma unroll
            for (int j = 0; j < NB; j++) sy -= A[(size_t)(kb + j) * N + i] * Y[kb + j];
            Y[i] = sy;
        }
        __syncthreads();
    }
    for (int i = t; i < n; i += LDLT_THREADS) d.x[i] = Y[i];
#ifdef MAM_LDLT_PROFILE
    __syncthreads();
    if (t == 0) d.red[7] += (double)(clock64() - tp0);
#endif
}

__global__ __launch_bounds__(256) void k_backsub(Dev d) {
    const int h = blockIdx.x * 256 + threadIdx.x;
    if (h >= d.L) return;
    double cl[3];
    for (int k = 0; k < 3; k++) cl[k] = d.b[6 * (size_t)d.Np + 3 * (size_t)h + k];
    for (int s = d.pe_off[h]; s < d.pe_off[h + 1]; s++) {
        const int e = d.pe_idx[s];
        const int hp = d.pose_h[d.edge_pose[e]];
        if (hp < 0) continue;
        const double* B = d.hpl + 18 * (size_t)e;
        for (int j = 0; j < 3; j++)
            for (int i = 0; i < 6; i++) cl[j] -= B[3 * i + j] * d.x[6 * (size_t)hp + i];
    }
    const double* Di = d.Dinv + 9 * (size_t)h;
    for (int i = 0; i < 3; i++)
        d.x[6 * (size_t)d.Np + 3 * (size_t)h + i] = Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1] + Di[3 * i + 2] * cl[2];
}

// Eigen Quaterniond(Matrix3d)
__device__ void rot_to_quat(const double m[9], double q[4]) {
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
        if (m[8] > m[3 * i + i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        q[i] = 0.5 * s;
        s = 0.5 / s;
        q[3] = (m[3 * k + j] - m[3 * j + k]) * s;
        q[j] = (m[3 * j + i] + m[3 * i + j]) * s;
        q[k] = (m[3 * k + i] + m[3 * i + k]) * s;
    }
}

__device__ void normalize_q(double q[4]) {
    if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}

// T <- exp(dx) * T (VertexSE3Expmap::oplusImpl) for non-fixed poses; X <- X + dx for points; fixed copied.
__global__ __launch_bounds__(256) void k_update(Dev d) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < d.P) {
        const double* T = d.pose + 7 * (size_t)i;
        double* O = d.pose_out + 7 * (size_t)i;
        const int h = d.pose_h[i];
        if (h < 0) {
            for (int k = 0; k < 7; k++) O[k] = T[k];
        } else {
            const double* u = d.x + 6 * (size_t)h;
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
            // exp * T
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
    }
    if (i < d.L) {
        const int p = d.hpoint[i];
        for (int k = 0; k < 3; k++) d.pt_out[3 * (size_t)p + k] = d.pt[3 * (size_t)p + k] + d.x[6 * (size_t)d.Np + 3 * (size_t)i + k];
    }
}

// sum_j x_j (lambda x_j + b_j) in fixed order (computeScale)
__global__ __launch_bounds__(RED) void k_scale(Dev d, double lambda) {
    __shared__ double s[RED];
    const int t = threadIdx.x;
    const int n = 6 * d.Np + 3 * d.L;
    double acc = 0.0;
    for (int j = t; j < n; j += RED) acc += d.x[j] * (lambda * d.x[j] + d.b[j]);
    s[t] = acc;
    __syncthreads();
    for (int o = RED / 2; o > 0; o >>= 1) {
        if (t < o) s[t] += s[t + o];
        __syncthreads();
    }
    if (t == 0) d.red[1] = s[0];
}

__global__ __launch_bounds__(256) void k_depth(Dev d, uint8_t* out) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= d.E) return;
    double Xc[3];
    map_point(d.pose + 7 * (size_t)d.edge_pose[e], d.pt + 3 * (size_t)d.edge_point[e], Xc);
    out[e] = Xc[2] > 0.0;
}

}  // namespace lba
}  // namespace mam

// ==================================================================================================== host
using mam::DevBuf;

struct mam_lba_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    size_t ldlt_lds_budget = 0;   // dynamic LDS the factorization may use (panel staging)
    mam::PinnedBuf staging;       // host mirror of the uploaded part of the arena (one copy per solve)
    mam::StageTimer timer{4};
    DevBuf<uint8_t> arena;
};

namespace {

struct Carver {
    uint8_t* base;
    size_t off = 0;
    template <typename T>
    T* take(size_t n) {
        T* p = reinterpret_cast<T*>(base + off);
        off += (n * sizeof(T) + 255) & ~(size_t)255;
        return p;
    }
};

template <typename T>
size_t sz(size_t n) { return (n * sizeof(T) + 255) & ~(size_t)255; }

}  // namespace

extern "C" {

int mam_lba_create(int device, mam_lba_ctx** out) {
    if (!out) return MAM_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    MAM_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) { mam::set_last_error("no such HIP device"); return MAM_ERR_ARG; }
    MAM_DEVICE_SCOPE(device);
    mam_lba_ctx* c = new mam_lba_ctx();
    c->device = device;
    // gfx950: 160 KB of LDS per workgroup; fall back to the 64 KB default if the opt-in is refused
    c->ldlt_lds_budget = 0;
    for (size_t budget : {(size_t)160 * 1024 - 4096, (size_t)64 * 1024 - 4096}) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::lba::k_ldlt<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)budget) == hipSuccess) {
            c->ldlt_lds_budget = budget;
            break;
        }
        (void)hipGetLastError();
    }
    // Highest stream priority: LocalMapping's solve shares the GPU with Tracking's full-chip launches, and its small
    // latency-bound kernels (and the host round trip of every LM trial) should not queue behind them.
    // MAM_LBA_PRIORITY=0 keeps the default priority.
    int least = 0, greatest = 0;
    const char* pe = std::getenv("MAM_LBA_PRIORITY");
    const bool prio = !(pe && pe[0] == '0') && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess;
    if (!(prio && hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest) == hipSuccess)) {
        (void)hipGetLastError();
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            delete c;
            return MAM_ERR_DEVICE;
        }
    }
    *out = c;
    return MAM_OK;
}

void mam_lba_destroy(mam_lba_ctx* c) {
    if (!c) return;
    ::mam::DeviceScope mam_dev_scope_(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

int mam_lba_set_profiling(mam_lba_ctx* c, int enable) {
    if (!c) return MAM_ERR_ARG;
    c->timer.reset(enable != 0);
    return MAM_OK;
}

int mam_lba_stage_times(mam_lba_ctx* c, double* ms_out, int64_t* launches_out) {
    if (!c) return MAM_ERR_ARG;
    c->timer.collect();
    for (int i = 0; i < 4; i++) {
        if (ms_out) ms_out[i] = c->timer.ms[i];
        if (launches_out) launches_out[i] = c->timer.n[i];
    }
    return MAM_OK;
}

int mam_lba_solve(mam_lba_ctx* c, const mam_lba_problem* p, const volatile uint8_t* stop_flag, mam_lba_result* r) {
    if (!c || !p || !r || p->n_poses < 0 || p->n_points < 0 || p->n_edges < 0 || !p->cams || p->n_cams < 1)
        return MAM_ERR_ARG;
    if ((p->n_poses > 0 && (!p->pose_id || !p->pose_fixed || !p->pose_q || !p->pose_t)) ||
        (p->n_points > 0 && (!p->point_id || !p->point_xyz)) ||
        (p->n_edges > 0 && (!p->edge_point || !p->edge_pose || !p->edge_obs || !p->edge_inv_sigma2)) ||
        !r->pose_q || !r->pose_t || (p->n_points > 0 && !r->point_xyz))
        return MAM_ERR_ARG;
    const int P = p->n_poses, L = p->n_points, E = p->n_edges;
    for (int e = 0; e < E; e++)
        if (p->edge_point[e] < 0 || p->edge_point[e] >= L || p->edge_pose[e] < 0 || p->edge_pose[e] >= P)
            return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
#ifdef MAM_LDLT_PROFILE
    const auto h_t0 = std::chrono::steady_clock::now();
#endif
    // ---- structure (sparse_optimizer.cpp:166-190): Hessian order = vertices sorted by id
    std::vector<int> po(P), pl(L);
    std::iota(po.begin(), po.end(), 0);
    std::iota(pl.begin(), pl.end(), 0);
    std::stable_sort(po.begin(), po.end(), [&](int a, int b) { return p->pose_id[a] < p->pose_id[b]; });
    std::stable_sort(pl.begin(), pl.end(), [&](int a, int b) { return p->point_id[a] < p->point_id[b]; });
    std::vector<int32_t> pose_h(P, -1), hpose, point_h(L, -1), hpoint;
    hpose.reserve(P);
    hpoint.reserve(L);
    for (int i : po)
        if (!p->pose_fixed[i]) { pose_h[i] = (int)hpose.size(); hpose.push_back(i); }
    for (int i : pl) { point_h[i] = (int)hpoint.size(); hpoint.push_back(i); }
    const int Np = (int)hpose.size();
    // per Hessian point / pose edge lists (counting sorts, edge order kept)
    std::vector<int32_t> pe_off(L + 1, 0), pe_idx(E), qe_off(Np + 1, 0), qe_idx;
    for (int e = 0; e < E; e++) {
        pe_off[point_h[p->edge_point[e]] + 1]++;
        const int h = pose_h[p->edge_pose[e]];
        if (h >= 0) qe_off[h + 1]++;
    }
    for (int h = 0; h < L; h++) pe_off[h + 1] += pe_off[h];
    for (int h = 0; h < Np; h++) qe_off[h + 1] += qe_off[h];
    qe_idx.resize(qe_off[Np]);
    {
        std::vector<int32_t> cp(pe_off.begin(), pe_off.end() - 1), cq(qe_off.begin(), qe_off.end() - 1);
        for (int e = 0; e < E; e++) {
            pe_idx[cp[point_h[p->edge_point[e]]]++] = e;
            const int h = pose_h[p->edge_pose[e]];
            if (h >= 0) qe_idx[cq[h]++] = e;
        }
    }
    // S block pairs (i1 <= i2, row-major; diagonal blocks always present) with their contributions in landmark
    // (Hessian point) order, then edge order within the landmark
    // every block of the upper triangle of S (g2o keeps only the non-empty ones; the empty ones are zero here)
    std::vector<int32_t> bp_ij;
    bp_ij.reserve((size_t)Np * (Np + 1));
    for (int a = 0; a < Np; a++)
        for (int b = a; b < Np; b++) { bp_ij.push_back(a); bp_ij.push_back(b); }
    const int nbp = (int)bp_ij.size() / 2;
    const int n = 6 * Np, nx = 6 * Np + 3 * L, npad = mam::lba::ldlt_pad(n);
    // ---- device arena: the uploaded inputs first (mirrored in pinned host memory, one copy), scratch after
    size_t bytes = sz<int32_t>(E) * 2 + sz<double>(2 * (size_t)E) + sz<double>(E) + sz<float>(4 * (size_t)p->n_cams) +
                   sz<int32_t>(P) * 2 + sz<int32_t>(Np) + sz<int32_t>(L) * 2 + sz<int32_t>(L + 1) + sz<int32_t>(E) +
                   sz<int32_t>(Np + 1) + sz<int32_t>(E) + sz<int32_t>((size_t)Np * L) +
                   sz<int32_t>(2 * (size_t)nbp) + 2 * sz<double>(7 * (size_t)P) + 2 * sz<double>(3 * (size_t)L) +
                   sz<double>(2 * (size_t)E) + sz<double>(21 * (size_t)E) + sz<double>(E) + sz<double>(18 * (size_t)E) * 2 +
                   sz<double>(6 * (size_t)E) + sz<double>(36 * (size_t)Np) + sz<double>(9 * (size_t)L) + sz<double>(nx) +
                   sz<double>(9 * (size_t)L) + sz<double>((size_t)npad * npad) + sz<double>(nx) + sz<double>(npad) + sz<double>(8) +
                   sz<double>(mam::lba::ldlt_ws_doubles(npad)) +
                   sz<int>(4) + sz<uint8_t>(E) * 2 + sz<double>((size_t)(E + 255) / 256 + 1) + 4096;
    if (int rc = c->arena.alloc(bytes)) return rc;
    if (int rc = c->staging.alloc(bytes)) return rc;
    Carver cv{c->arena.p};
    uint8_t* const host_base = c->staging.p;
    mam::lba::Dev d{};
    d.P = P; d.L = L; d.E = E; d.Np = Np; d.nbp = nbp; d.npad = npad; d.delta = p->huber_delta;
    hipStream_t s = c->stream;
    // carve a device array and fill its pinned mirror
    auto put = [&](auto* src, size_t count) {
        using T = std::remove_const_t<std::remove_pointer_t<decltype(src)>>;
        T* dst = cv.take<T>(count);
        if (count) std::memcpy(host_base + (reinterpret_cast<uint8_t*>(dst) - c->arena.p), src, count * sizeof(T));
        return dst;
    };
    d.edge_point = put(p->edge_point, E);
    d.edge_pose = put(p->edge_pose, E);
    d.edge_obs = put(p->edge_obs, 2 * (size_t)E);
    d.edge_w = put(p->edge_inv_sigma2, E);
    d.active = p->edge_active ? put(p->edge_active, E) : nullptr;
    d.cams = put(p->cams, 4 * (size_t)p->n_cams);
    {
        const int32_t* pcm = put(p->pose_cam ? p->pose_cam : pose_h.data(), P);
        d.pose_cam = p->pose_cam ? pcm : nullptr;
    }
    d.pose_h = put(pose_h.data(), P);
    d.hpose = put(hpose.data(), Np);
    d.hpoint = put(hpoint.data(), L);
    d.point_h = put(point_h.data(), L);
    d.pe_off = put(pe_off.data(), L + 1);
    d.pe_idx = put(pe_idx.data(), E);
    d.qe_off = put(qe_off.data(), Np + 1);
    d.qe_idx = put(qe_idx.data(), qe_idx.size());
    d.bp_ij = put(bp_ij.data(), 2 * (size_t)nbp);
    // state: poses packed [q t], SE3Quat(q, t) normalises on construction
    std::vector<double> pose0(7 * (size_t)P);
    for (int i = 0; i < P; i++) {
        double q[4] = {p->pose_q[4 * i], p->pose_q[4 * i + 1], p->pose_q[4 * i + 2], p->pose_q[4 * i + 3]};
        if (q[3] < 0) for (double& v : q) v = -v;
        const double nq = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (int k = 0; k < 4; k++) pose0[7 * i + k] = q[k] / nq;
        for (int k = 0; k < 3; k++) pose0[7 * i + 4 + k] = p->pose_t[3 * i + k];
    }
    double* poseA = put(pose0.data(), 7 * (size_t)P);
    double* ptA = put(p->point_xyz, 3 * (size_t)L);
    const size_t upload = cv.off;
#ifdef MAM_LDLT_PROFILE
    const auto h_t1 = std::chrono::steady_clock::now();
#endif
    MAM_HIP(hipMemcpyAsync(c->arena.p, host_base, upload, hipMemcpyHostToDevice, s));
    d.eidx = cv.take<int32_t>((size_t)Np * L);
    if ((size_t)Np * L > 0) {
        MAM_HIP(hipMemsetAsync(d.eidx, 0xFF, sizeof(int32_t) * (size_t)Np * L, s));
        if (E > 0) hipLaunchKernelGGL(mam::lba::k_eidx, dim3((E + 255) / 256), dim3(256), 0, s, d);
    }
    double* poseB = cv.take<double>(7 * (size_t)P);
    double* ptB = cv.take<double>(3 * (size_t)L);
    d.err = cv.take<double>(2 * (size_t)E);
    d.jac = cv.take<double>(21 * (size_t)E);
    d.rho0 = cv.take<double>(E);
    d.part = cv.take<double>((size_t)(E + 255) / 256 + 1);
    d.hpl = cv.take<double>(18 * (size_t)E);
    d.bdinv = cv.take<double>(18 * (size_t)E);
    d.coef = cv.take<double>(6 * (size_t)E);
    d.Hpp = cv.take<double>(36 * (size_t)Np);
    d.Hll = cv.take<double>(9 * (size_t)L);
    d.b = cv.take<double>(nx);
    d.Dinv = cv.take<double>(9 * (size_t)L);
    d.S = cv.take<double>((size_t)npad * npad);
    d.x = cv.take<double>(nx);
    d.bs = cv.take<double>(npad);
    d.ws = cv.take<double>(mam::lba::ldlt_ws_doubles(npad));
    d.red = cv.take<double>(8);
    MAM_HIP(hipMemsetAsync(d.red, 0, sizeof(double) * 8, s));
    d.flag = cv.take<int>(4);
    uint8_t* depth = cv.take<uint8_t>(E);
    MAM_HIP(hipMemsetAsync(d.x, 0, sizeof(double) * nx, s));
    if (npad > 0) MAM_HIP(hipMemsetAsync(d.bs, 0, sizeof(double) * npad, s));

    const int gE = (E + 255) / 256, gL = (L + 255) / 256, gPL = (std::max(P, L) + 255) / 256;
    double* cur_pose = poseA; double* cur_pt = ptA;
    double* tr_pose = poseB;  double* tr_pt = ptB;
    auto state = [&](const double* pose, const double* pt, double* opose, double* opt) {
        d.pose = pose; d.pt = pt; d.pose_out = opose; d.pt_out = opt;
    };
    double h_red[3];
    auto chi_of = [&](const double* pose, const double* pt, bool jac, double* out_chi) -> int {
        state(pose, pt, tr_pose, tr_pt);
        if (E > 0) hipLaunchKernelGGL(mam::lba::k_linearize, dim3(gE), dim3(256), 0, s, d, jac ? 1 : 0);
        hipLaunchKernelGGL(mam::lba::k_reduce_chi, dim3(1), dim3(mam::lba::RED), 0, s, d, 0);
        MAM_HIP(hipMemcpyAsync(h_red, d.red, sizeof(double), hipMemcpyDeviceToHost, s));
        MAM_HIP(hipStreamSynchronize(s));
        *out_chi = h_red[0];
        return MAM_OK;
    };
    auto stopped = [&]() { return stop_flag && *stop_flag; };

    double chi0 = 0;
    if (int rc = chi_of(cur_pose, cur_pt, false, &chi0)) return rc;
    r->initial_chi2 = chi0;
    double currentLambda = -1.0, ni = 2.0, acceptedChi = chi0;
    int nBad = 0, trials = 0, its = 0;
    bool ok = Np + L > 0;
    for (int it = 0; it < p->iterations && !stopped() && ok; it++) {
        double currentChi;
        {
            mam::StageTimer::Scope sc(&c->timer, s, 0);
            state(cur_pose, cur_pt, tr_pose, tr_pt);
            if (E > 0) hipLaunchKernelGGL(mam::lba::k_linearize, dim3(gE), dim3(256), 0, s, d, 1);
            hipLaunchKernelGGL(mam::lba::k_reduce_chi, dim3(1), dim3(mam::lba::RED), 0, s, d, 0);
            if (L > 0) hipLaunchKernelGGL(mam::lba::k_point_sys, dim3((L + 63) / 64), dim3(64), 0, s, d);
            if (Np > 0) hipLaunchKernelGGL(mam::lba::k_pose_sys, dim3(Np), dim3(64), 0, s, d);
            hipLaunchKernelGGL(mam::lba::k_max_diag, dim3(1), dim3(mam::lba::RED), 0, s, d);
        }
        if (it == 0) {
            // lambda init needs max diag(H); afterwards the iteration-start chi2 is, bit for bit, the chi2 of the
            // trial that was just accepted (same kernels on the same state), so no round trip is needed
            MAM_HIP(hipMemcpyAsync(h_red, d.red, 3 * sizeof(double), hipMemcpyDeviceToHost, s));
            MAM_HIP(hipStreamSynchronize(s));
            currentChi = h_red[0];
            currentLambda = 1e-5 * h_red[2];
            ni = 2;
            nBad = 0;
        } else {
            currentChi = acceptedChi;
        }
        const double iniChi = currentChi;
        double rho = 0;
        int qmax = 0;
        do {
            {
                mam::StageTimer::Scope sc(&c->timer, s, 1);
                if (L > 0) hipLaunchKernelGGL(mam::lba::k_schur_prep, dim3((L + 63) / 64), dim3(64), 0, s, d, currentLambda);
                if (E > 0) hipLaunchKernelGGL(mam::lba::k_schur_edge, dim3(gE), dim3(256), 0, s, d);
                // the factorization leaves fill-in in S: clear the whole matrix before the blocks are rewritten
                if (npad > 0) MAM_HIP(hipMemsetAsync(d.S, 0, sizeof(double) * (size_t)npad * npad, s));
                if (nbp > 0) hipLaunchKernelGGL(mam::lba::k_schur_blk, dim3(nbp), dim3(64), 0, s, d, currentLambda);
                if (Np > 0) hipLaunchKernelGGL(mam::lba::k_schur_rhs, dim3(Np), dim3(64), 0, s, d);
            }
            {
                mam::StageTimer::Scope sc(&c->timer, s, 2);
                MAM_HIP(hipMemsetAsync(d.flag, 0, sizeof(int), s));
                if (Np > 0) {
                    const size_t lds = mam::lba::ldlt_lds_bytes(npad);
                    if (lds <= c->ldlt_lds_budget)
                        hipLaunchKernelGGL(mam::lba::k_ldlt<true>, dim3(1), dim3(mam::lba::LDLT_THREADS), lds, s, d);
                    else
                        hipLaunchKernelGGL(mam::lba::k_ldlt<false>, dim3(1), dim3(mam::lba::LDLT_THREADS), 0, s, d);
                }
            }
            {
                mam::StageTimer::Scope sc(&c->timer, s, 3);
                if (L > 0) hipLaunchKernelGGL(mam::lba::k_backsub, dim3(gL), dim3(256), 0, s, d);
                state(cur_pose, cur_pt, tr_pose, tr_pt);
                if (std::max(P, L) > 0) hipLaunchKernelGGL(mam::lba::k_update, dim3(gPL), dim3(256), 0, s, d);
                // chi2 of the trial state (errors kept: chi2() reads the last computeActiveErrors)
                state(tr_pose, tr_pt, tr_pose, tr_pt);
                if (E > 0) hipLaunchKernelGGL(mam::lba::k_linearize, dim3(gE), dim3(256), 0, s, d, 0);
                hipLaunchKernelGGL(mam::lba::k_reduce_chi, dim3(1), dim3(mam::lba::RED), 0, s, d, 0);
                hipLaunchKernelGGL(mam::lba::k_scale, dim3(1), dim3(mam::lba::RED), 0, s, d, currentLambda);
            }
            int fail = 0;
            MAM_HIP(hipMemcpyAsync(h_red, d.red, 2 * sizeof(double), hipMemcpyDeviceToHost, s));
            MAM_HIP(hipMemcpyAsync(&fail, d.flag, sizeof(int), hipMemcpyDeviceToHost, s));
            MAM_HIP(hipStreamSynchronize(s));
            double tempChi = h_red[0];
            if (fail) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = h_red[1] + 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                currentLambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
                acceptedChi = tempChi;
                std::swap(cur_pose, tr_pose);   // accept: discardTop
                std::swap(cur_pt, tr_pt);
            } else {
                currentLambda *= ni;             // reject: pop
                ni *= 2;
            }
            qmax++;
            trials++;
        } while (rho < 0 && qmax < 10 && !stopped());
        its++;
        bool term = false;
        if (qmax == 10 || rho == 0) term = true;
        else {
            if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
            else nBad = 0;
            if (nBad >= 3) term = true;
        }
        ok = !term;
    }
    MAM_HIP(hipGetLastError());
#ifdef MAM_LDLT_PROFILE
    {
        double ph[4];
        MAM_HIP(hipMemcpy(ph, d.red + 4, sizeof(ph), hipMemcpyDeviceToHost));
        const auto h_t2 = std::chrono::steady_clock::now();
        fprintf(stderr, "ldlt cycles: diag+trailing-rest %.0f panel %.0f next-column %.0f subst %.0f (trials %d); host setup %.3f ms, "
                "loop %.3f ms\n", ph[0], ph[1], ph[2], ph[3], trials,
                std::chrono::duration<double, std::milli>(h_t1 - h_t0).count(),
                std::chrono::duration<double, std::milli>(h_t2 - h_t1).count());
    }
#endif
    // ---- results
    std::vector<double> pose_h_out(7 * (size_t)P);
    if (P) MAM_HIP(hipMemcpyAsync(pose_h_out.data(), cur_pose, sizeof(double) * 7 * P, hipMemcpyDeviceToHost, s));
    if (L) MAM_HIP(hipMemcpyAsync(r->point_xyz, cur_pt, sizeof(double) * 3 * L, hipMemcpyDeviceToHost, s));
    if (r->edge_chi2 && E) {
        // chi2() = e^T Omega e of the last computed errors
        std::vector<double> err(2 * (size_t)E);
        MAM_HIP(hipMemcpyAsync(err.data(), d.err, sizeof(double) * 2 * E, hipMemcpyDeviceToHost, s));
        MAM_HIP(hipStreamSynchronize(s));
        for (int e = 0; e < E; e++) {
            if (p->edge_active && !p->edge_active[e]) continue;   // not computed at level 0: left to the caller
            const double w = p->edge_inv_sigma2[e], e0 = err[2 * e], e1 = err[2 * e + 1];
            r->edge_chi2[e] = e0 * (w * e0) + e1 * (w * e1);
        }
    }
    state(cur_pose, cur_pt, tr_pose, tr_pt);
    if (r->edge_depth_ok && E) {
        hipLaunchKernelGGL(mam::lba::k_depth, dim3(gE), dim3(256), 0, s, d, depth);
        MAM_HIP(hipMemcpyAsync(r->edge_depth_ok, depth, E, hipMemcpyDeviceToHost, s));
    }
    MAM_HIP(hipStreamSynchronize(s));
    for (int i = 0; i < P; i++) {
        for (int k = 0; k < 4; k++) r->pose_q[4 * i + k] = pose_h_out[7 * i + k];
        for (int k = 0; k < 3; k++) r->pose_t[3 * i + k] = pose_h_out[7 * i + 4 + k];
    }
    r->final_chi2 = acceptedChi;   // activeRobustChi2 of the final state: the last accepted trial's (or initial) chi2
    r->iterations = its;
    r->lm_trials = trials;
    r->status = stopped() ? 1 : 0;
    return MAM_OK;
}

}  // extern "C"
