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
#include <cmath>
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
    const int32_t* point_h;      // unused on device (points are indexed by Hessian order directly)
    const int32_t* hpoint;       // Hessian point -> point
    const int32_t* pe_off;       // per Hessian point: edge segment [pe_off[h], pe_off[h+1]) into pe_idx
    const int32_t* pe_idx;
    const int32_t* qe_off;       // per Hessian pose: edges
    const int32_t* qe_idx;
    const int32_t* bp_off;       // per S block pair: contributions
    const int32_t* bp_ea;
    const int32_t* bp_ec;
    const int32_t* bp_ij;        // (i1, i2) per block pair
    int nbp;
    double delta;
    // state
    const double* pose;          // [P][7] q(xyzw) t
    const double* pt;            // [L][3]
    double* pose_out;            // trial
    double* pt_out;
    // per edge
    double* err;                 // [E][2]
    double* jac;                 // [E][21]: A(6) B(12) orr(2) wo(1)
    double* rho0;                // [E]
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
    if (e <= dsqr) { *r0 = e; *r1 = 1.0; }
    else {
        const double s = sqrt(e);
        *r0 = 2 * s * delta - dsqr;
        *r1 = delta / s;
    }
}

// ---- per edge: error, robust weight, Jacobians (EdgeSE3ProjectXYZ)
__global__ __launch_bounds__(256) void k_linearize(Dev d, int want_jac) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= d.E) return;
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
    const double w = d.edge_w[e];
    const double chi = e0 * (w * e0) + e1 * (w * e1);
    double r0, r1;
    huber(chi, d.delta, &r0, &r1);
    d.rho0[e] = r0;
    if (!want_jac) return;
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
}

// ---- per point: H_ll, b_l, per-edge H_pl
__global__ __launch_bounds__(256) void k_point_sys(Dev d) {
    const int h = blockIdx.x * 256 + threadIdx.x;
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
        if (d.pose_h[d.edge_pose[e]] >= 0) {
            double* hp = d.hpl + 18 * (size_t)e;
            for (int a = 0; a < 6; a++)
                for (int c = 0; c < 3; c++) hp[3 * a + c] = j[6 + a] * wo * j[c] + j[12 + a] * wo * j[3 + c];
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

// ---- fixed-order sum of rho0 (and max diag) in one workgroup
__global__ __launch_bounds__(1024) void k_reduce_chi(Dev d, int slot) {
    __shared__ double s[1024];
    const int t = threadIdx.x;
    double acc = 0.0;
    for (int e = t; e < d.E; e += 1024) acc += d.rho0[e];
    s[t] = acc;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (t < o) s[t] += s[t + o];
        __syncthreads();
    }
    if (t == 0) d.red[slot] = s[0];
}

__global__ __launch_bounds__(1024) void k_max_diag(Dev d) {
    __shared__ double s[1024];
    const int t = threadIdx.x;
    double m = 0.0;
    for (int i = t; i < 6 * d.Np; i += 1024) m = fmax(m, fabs(d.Hpp[36 * (size_t)(i / 6) + 7 * (i % 6)]));
    for (int i = t; i < 3 * d.L; i += 1024) m = fmax(m, fabs(d.Hll[9 * (size_t)(i / 3) + 4 * (i % 3)]));
    s[t] = m;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
        if (t < o) s[t] = fmax(s[t], s[t + o]);
        __syncthreads();
    }
    if (t == 0) d.red[2] = s[0];
}

// ---- Schur
__global__ __launch_bounds__(256) void k_schur_prep(Dev d, double lambda) {
    const int h = blockIdx.x * 256 + threadIdx.x;
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
    const double* bl = d.b + 6 * (size_t)d.Np + 3 * (size_t)h;
    double db[3];
    for (int i = 0; i < 3; i++) db[i] = Di[3 * i] * bl[0] + Di[3 * i + 1] * bl[1] + Di[3 * i + 2] * bl[2];
    for (int s = d.pe_off[h]; s < d.pe_off[h + 1]; s++) {
        const int e = d.pe_idx[s];
        if (d.pose_h[d.edge_pose[e]] < 0) continue;
        const double* B = d.hpl + 18 * (size_t)e;
        double* o = d.bdinv + 18 * (size_t)e;
        double* cf = d.coef + 6 * (size_t)e;
        for (int i = 0; i < 6; i++) {
            for (int j = 0; j < 3; j++) o[3 * i + j] = B[3 * i] * Di[j] + B[3 * i + 1] * Di[3 + j] + B[3 * i + 2] * Di[6 + j];
            cf[i] = B[3 * i] * db[0] + B[3 * i + 1] * db[1] + B[3 * i + 2] * db[2];
        }
    }
}

__global__ __launch_bounds__(64) void k_schur_blk(Dev d, double lambda) {
    const int bp = blockIdx.x, lane = threadIdx.x;
    const int i1 = d.bp_ij[2 * bp], i2 = d.bp_ij[2 * bp + 1];
    double acc[36];
#pragma unroll
    for (int k = 0; k < 36; k++) acc[k] = 0.0;
    for (int s = d.bp_off[bp] + lane; s < d.bp_off[bp + 1]; s += 64) {
        const double* W = d.bdinv + 18 * (size_t)d.bp_ea[s];
        const double* B = d.hpl + 18 * (size_t)d.bp_ec[s];
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
        const int n = 6 * d.Np;
        d.S[(size_t)(6 * i1 + r) * n + 6 * i2 + c] = out;
        d.S[(size_t)(6 * i2 + c) * n + 6 * i1 + r] = out;
    }
}

__global__ __launch_bounds__(64) void k_schur_rhs(Dev d) {
    const int h = blockIdx.x, lane = threadIdx.x;
    if (lane >= 6) return;
    double acc = d.b[6 * (size_t)h + lane];
    for (int s = d.qe_off[h]; s < d.qe_off[h + 1]; s++) acc -= d.coef[6 * (size_t)d.qe_idx[s] + lane];
    d.bs[6 * (size_t)h + lane] = acc;
}

// ---- dense LDL^T solve of S x = bs, one workgroup, blocked right-looking with NB = 16 column panels.
// S holds the full symmetric matrix. Per panel: (1) wave 0 factors the 16x16 diagonal block in registers
// (lane i owns row i, columns broadcast by shuffles); (2) every thread forward-solves panel rows
// L21 = A21 L11^-T D^-1 and keeps W = L21 D in the (dead) upper triangle; (3) the trailing lower triangle
// is updated A22 -= L21 W^T in 4x4 register tiles. flag[0] = 1 on an exact zero pivot (the failure rule of
// Eigen's SimplicialLDLT). Then blocked forward / diagonal / backward substitution.
constexpr int NB = 16;

__global__ __launch_bounds__(1024) void k_ldlt(Dev d) {
    const int n = 6 * d.Np;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    double* A = d.S;
    __shared__ double Ld[NB * NB];
    __shared__ double dk[NB];
    __shared__ int fail;
    if (t == 0) fail = 0;
    for (int kb = 0; kb < n; kb += NB) {
        const int nb = min(NB, n - kb);
        // (1) diagonal block
        if (wid == 0) {
            double row[NB];
#pragma unroll
            for (int c = 0; c < NB; c++) row[c] = (lane < nb && c < nb) ? A[(size_t)(kb + lane) * n + kb + c] : 0.0;
            double dloc[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) {
                if (j < nb) {
                    // d_j = a_jj - sum_k L_jk^2 d_k  (lane j holds row j)
                    double s = row[j];
#pragma unroll
                    for (int k = 0; k < NB; k++)
                        if (k < j) s -= row[k] * row[k] * dloc[k];
                    const double dj = __shfl(s, j, 64);
                    dloc[j] = dj;
                    // L_ij = (a_ij - sum_k L_ik L_jk d_k) / d_j for i > j
                    double lj[NB];
#pragma unroll
                    for (int k = 0; k < NB; k++) lj[k] = __shfl(row[k], j, 64);
                    if (lane > j && lane < nb) {
                        double v = row[j];
#pragma unroll
                        for (int k = 0; k < NB; k++)
                            if (k < j) v -= row[k] * lj[k] * dloc[k];
                        row[j] = dj != 0.0 ? v / dj : 0.0;
                    }
                } else {
                    dloc[j] = 1.0;
                }
            }
            if (lane < nb) {
#pragma unroll
                for (int c = 0; c < NB; c++) Ld[lane * NB + c] = row[c];
                dk[lane] = dloc[lane < NB ? lane : 0];
                if (dloc[lane] == 0.0) fail = 1;
            }
        }
        __syncthreads();
        for (int i = t; i < nb * nb; i += 1024) {
            const int r = i / nb, c = i % nb;
            if (r > c) A[(size_t)(kb + r) * n + kb + c] = Ld[r * NB + c];
            else if (r == c) A[(size_t)(kb + r) * n + kb + c] = dk[r];
        }
        // (2) panel rows
        for (int i = kb + nb + t; i < n; i += 1024) {
            double w[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) {
                if (j < nb) {
                    double s = A[(size_t)i * n + kb + j];
#pragma unroll
                    for (int k = 0; k < NB; k++)
                        if (k < j) s -= w[k] * Ld[j * NB + k];
                    w[j] = s;
                }
            }
#pragma unroll
            for (int j = 0; j < NB; j++) {
                if (j < nb) {
                    A[(size_t)i * n + kb + j] = dk[j] != 0.0 ? w[j] / dk[j] : 0.0;   // L21
                    A[(size_t)(kb + j) * n + i] = w[j];                               // W^T (upper, dead)
                }
            }
        }
        __syncthreads();
        // (3) trailing update, 4x4 register tiles over the lower triangle of the m x m trailing block
        const int m = n - kb - nb;
        const int T = (m + 3) / 4;
        const int ntile = T * (T + 1) / 2;
        for (int q = t; q < ntile; q += 1024) {
            int tr = (int)((sqrt(8.0 * (double)q + 1.0) - 1.0) * 0.5);
            while (tr * (tr + 1) / 2 > q) tr--;
            while ((tr + 1) * (tr + 2) / 2 <= q) tr++;
            const int tc = q - tr * (tr + 1) / 2;
            const int r0 = kb + nb + 4 * tr, c0 = kb + nb + 4 * tc;
            double acc[4][4];
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int b = 0; b < 4; b++) acc[a][b] = 0.0;
            for (int k = 0; k < nb; k++) {
                double lr[4], wc[4];
#pragma unroll
                for (int a = 0; a < 4; a++) {
                    lr[a] = (r0 + a < n) ? A[(size_t)(r0 + a) * n + kb + k] : 0.0;
                    wc[a] = (c0 + a < n) ? A[(size_t)(kb + k) * n + c0 + a] : 0.0;
                }
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int b = 0; b < 4; b++) acc[a][b] += lr[a] * wc[b];
            }
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const int gi = r0 + a, gj = c0 + b;
                    if (gi < n && gj < n && gj <= gi) A[(size_t)gi * n + gj] -= acc[a][b];
                }
        }
        __syncthreads();
    }
    if (t == 0) d.flag[0] = fail;
    __syncthreads();
    if (fail) return;
    // blocked substitution: L y = bs; y /= D; L^T x = y
    double* y = d.x;
    for (int i = t; i < n; i += 1024) y[i] = d.bs[i];
    __syncthreads();
    for (int kb = 0; kb < n; kb += NB) {
        const int nb = min(NB, n - kb);
        if (wid == 0) {
            // unit-lower triangular solve of the 16-row block in one wave
            double v = lane < nb ? y[kb + lane] : 0.0;
            for (int j = 0; j < nb; j++) {
                const double yj = __shfl(v, j, 64);
                if (lane > j && lane < nb) v -= A[(size_t)(kb + lane) * n + kb + j] * yj;
            }
            if (lane < nb) y[kb + lane] = v;
        }
        __syncthreads();
        for (int i = kb + nb + t; i < n; i += 1024) {
            double s = y[i];
            for (int j = 0; j < nb; j++) s -= A[(size_t)i * n + kb + j] * y[kb + j];
            y[i] = s;
        }
        __syncthreads();
    }
    for (int i = t; i < n; i += 1024) y[i] /= A[(size_t)i * n + i];
    __syncthreads();
    const int nblk = (n + NB - 1) / NB;
    for (int bi = nblk - 1; bi >= 0; bi--) {
        const int kb = bi * NB, nb = min(NB, n - kb);
        if (wid == 0) {
            // unit-upper (L^T) solve of the block: x_i = y_i - sum_{j>i} L_ji x_j
            double v = lane < nb ? y[kb + lane] : 0.0;
            for (int j = nb - 1; j >= 0; j--) {
                const double xj = __shfl(v, j, 64);
                if (lane < j) v -= A[(size_t)(kb + j) * n + kb + lane] * xj;
            }
            if (lane < nb) y[kb + lane] = v;
        }
        __syncthreads();
        for (int i = t; i < kb; i += 1024) {
            double s = y[i];
            for (int j = 0; j < nb; j++) s -= A[(size_t)(kb + j) * n + i] * y[kb + j];
            y[i] = s;
        }
        __syncthreads();
    }
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
__global__ __launch_bounds__(1024) void k_scale(Dev d, double lambda) {
    __shared__ double s[1024];
    const int t = threadIdx.x;
    const int n = 6 * d.Np + 3 * d.L;
    double acc = 0.0;
    for (int j = t; j < n; j += 1024) acc += d.x[j] * (lambda * d.x[j] + d.b[j]);
    s[t] = acc;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
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
    MAM_HIP(hipSetDevice(device));
    mam_lba_ctx* c = new mam_lba_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return MAM_ERR_DEVICE;
    }
    *out = c;
    return MAM_OK;
}

void mam_lba_destroy(mam_lba_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
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
    MAM_HIP(hipSetDevice(c->device));
    // ---- structure (sparse_optimizer.cpp:166-190): Hessian order = vertices sorted by id
    std::vector<int> po(P), pl(L);
    std::iota(po.begin(), po.end(), 0);
    std::iota(pl.begin(), pl.end(), 0);
    std::stable_sort(po.begin(), po.end(), [&](int a, int b) { return p->pose_id[a] < p->pose_id[b]; });
    std::stable_sort(pl.begin(), pl.end(), [&](int a, int b) { return p->point_id[a] < p->point_id[b]; });
    std::vector<int32_t> pose_h(P, -1), hpose, point_h(L, -1), hpoint;
    for (int i : po)
        if (!p->pose_fixed[i]) { pose_h[i] = (int)hpose.size(); hpose.push_back(i); }
    for (int i : pl) { point_h[i] = (int)hpoint.size(); hpoint.push_back(i); }
    const int Np = (int)hpose.size();
    std::vector<std::vector<int>> pe(L);
    for (int e = 0; e < E; e++) pe[point_h[p->edge_point[e]]].push_back(e);
    std::vector<int32_t> pe_off(L + 1, 0), pe_idx;
    for (int h = 0; h < L; h++) { pe_idx.insert(pe_idx.end(), pe[h].begin(), pe[h].end()); pe_off[h + 1] = (int)pe_idx.size(); }
    std::vector<std::vector<int>> qe(Np);
    for (int e = 0; e < E; e++) {
        const int h = pose_h[p->edge_pose[e]];
        if (h >= 0) qe[h].push_back(e);
    }
    std::vector<int32_t> qe_off(Np + 1, 0), qe_idx;
    for (int h = 0; h < Np; h++) { qe_idx.insert(qe_idx.end(), qe[h].begin(), qe[h].end()); qe_off[h + 1] = (int)qe_idx.size(); }
    // S block pairs (i1 <= i2) with their contributions in landmark (Hessian point) order
    std::vector<std::vector<std::pair<int, int>>> blk((size_t)Np * Np);
    for (int h = 0; h < L; h++) {
        const std::vector<int>& Es = pe[h];
        for (int ea : Es) {
            const int ha = pose_h[p->edge_pose[ea]];
            if (ha < 0) continue;
            for (int ec : Es) {
                const int hc = pose_h[p->edge_pose[ec]];
                if (hc < 0 || hc < ha) continue;
                blk[(size_t)ha * Np + hc].push_back({ea, ec});
            }
        }
    }
    std::vector<int32_t> bp_off(1, 0), bp_ea, bp_ec, bp_ij;
    for (int a = 0; a < Np; a++)
        for (int b = a; b < Np; b++) {
            const auto& v = blk[(size_t)a * Np + b];
            if (v.empty() && a != b) continue;
            for (auto& pr : v) { bp_ea.push_back(pr.first); bp_ec.push_back(pr.second); }
            bp_off.push_back((int)bp_ea.size());
            bp_ij.push_back(a);
            bp_ij.push_back(b);
        }
    const int nbp = (int)bp_ij.size() / 2;
    const int n = 6 * Np, nx = 6 * Np + 3 * L;
    // ---- device arena
    size_t bytes = sz<int32_t>(E) * 2 + sz<double>(2 * (size_t)E) + sz<double>(E) + sz<float>(4 * (size_t)p->n_cams) +
                   sz<int32_t>(P) * 2 + sz<int32_t>(Np) + sz<int32_t>(L) + sz<int32_t>(L + 1) + sz<int32_t>(E) +
                   sz<int32_t>(Np + 1) + sz<int32_t>(E) + sz<int32_t>(nbp + 1) + sz<int32_t>(bp_ea.size()) * 2 +
                   sz<int32_t>(2 * (size_t)nbp) + 2 * sz<double>(7 * (size_t)P) + 2 * sz<double>(3 * (size_t)L) +
                   sz<double>(2 * (size_t)E) + sz<double>(21 * (size_t)E) + sz<double>(E) + 2 * sz<double>(18 * (size_t)E) +
                   sz<double>(6 * (size_t)E) + sz<double>(36 * (size_t)Np) + sz<double>(9 * (size_t)L) + sz<double>(nx) +
                   sz<double>(9 * (size_t)L) + sz<double>((size_t)n * n) + sz<double>(nx) + sz<double>(n) + sz<double>(8) +
                   sz<int>(4) + sz<uint8_t>(E) + 4096;
    if (int rc = c->arena.alloc(bytes)) return rc;
    Carver cv{c->arena.p};
    mam::lba::Dev d{};
    d.P = P; d.L = L; d.E = E; d.Np = Np; d.nbp = nbp; d.delta = p->huber_delta;
    hipStream_t s = c->stream;
    auto up = [&](auto* dst, const auto* src, size_t count) -> int {
        if (count) MAM_HIP(hipMemcpyAsync((void*)dst, (const void*)src, count * sizeof(*src), hipMemcpyHostToDevice, s));
        return MAM_OK;
    };
    int32_t* ep = cv.take<int32_t>(E); if (int rc = up(ep, p->edge_point, E)) return rc; d.edge_point = ep;
    int32_t* eq = cv.take<int32_t>(E); if (int rc = up(eq, p->edge_pose, E)) return rc; d.edge_pose = eq;
    double* eo = cv.take<double>(2 * (size_t)E); if (int rc = up(eo, p->edge_obs, 2 * (size_t)E)) return rc; d.edge_obs = eo;
    double* ew = cv.take<double>(E); if (int rc = up(ew, p->edge_inv_sigma2, E)) return rc; d.edge_w = ew;
    float* cams = cv.take<float>(4 * (size_t)p->n_cams); if (int rc = up(cams, p->cams, 4 * (size_t)p->n_cams)) return rc; d.cams = cams;
    int32_t* pc = cv.take<int32_t>(P);
    if (p->pose_cam) { if (int rc = up(pc, p->pose_cam, P)) return rc; d.pose_cam = pc; } else d.pose_cam = nullptr;
    int32_t* ph = cv.take<int32_t>(P); if (int rc = up(ph, pose_h.data(), P)) return rc; d.pose_h = ph;
    int32_t* hp = cv.take<int32_t>(Np); if (int rc = up(hp, hpose.data(), Np)) return rc; d.hpose = hp;
    int32_t* hl = cv.take<int32_t>(L); if (int rc = up(hl, hpoint.data(), L)) return rc; d.hpoint = hl;
    int32_t* peo = cv.take<int32_t>(L + 1); if (int rc = up(peo, pe_off.data(), L + 1)) return rc; d.pe_off = peo;
    int32_t* pei = cv.take<int32_t>(E); if (int rc = up(pei, pe_idx.data(), pe_idx.size())) return rc; d.pe_idx = pei;
    int32_t* qeo = cv.take<int32_t>(Np + 1); if (int rc = up(qeo, qe_off.data(), Np + 1)) return rc; d.qe_off = qeo;
    int32_t* qei = cv.take<int32_t>(E); if (int rc = up(qei, qe_idx.data(), qe_idx.size())) return rc; d.qe_idx = qei;
    int32_t* bpo = cv.take<int32_t>(nbp + 1); if (int rc = up(bpo, bp_off.data(), nbp + 1)) return rc; d.bp_off = bpo;
    int32_t* bpa = cv.take<int32_t>(bp_ea.size()); if (int rc = up(bpa, bp_ea.data(), bp_ea.size())) return rc; d.bp_ea = bpa;
    int32_t* bpc = cv.take<int32_t>(bp_ec.size()); if (int rc = up(bpc, bp_ec.data(), bp_ec.size())) return rc; d.bp_ec = bpc;
    int32_t* bij = cv.take<int32_t>(2 * (size_t)nbp); if (int rc = up(bij, bp_ij.data(), bp_ij.size())) return rc; d.bp_ij = bij;
    // state: poses packed [q t], SE3Quat(q, t) normalises on construction
    std::vector<double> pose0(7 * (size_t)P);
    for (int i = 0; i < P; i++) {
        double q[4] = {p->pose_q[4 * i], p->pose_q[4 * i + 1], p->pose_q[4 * i + 2], p->pose_q[4 * i + 3]};
        if (q[3] < 0) for (double& v : q) v = -v;
        const double nq = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (int k = 0; k < 4; k++) pose0[7 * i + k] = q[k] / nq;
        for (int k = 0; k < 3; k++) pose0[7 * i + 4 + k] = p->pose_t[3 * i + k];
    }
    double* poseA = cv.take<double>(7 * (size_t)P);
    double* poseB = cv.take<double>(7 * (size_t)P);
    double* ptA = cv.take<double>(3 * (size_t)L);
    double* ptB = cv.take<double>(3 * (size_t)L);
    if (int rc = up(poseA, pose0.data(), pose0.size())) return rc;
    if (int rc = up(ptA, p->point_xyz, 3 * (size_t)L)) return rc;
    d.err = cv.take<double>(2 * (size_t)E);
    d.jac = cv.take<double>(21 * (size_t)E);
    d.rho0 = cv.take<double>(E);
    d.hpl = cv.take<double>(18 * (size_t)E);
    d.bdinv = cv.take<double>(18 * (size_t)E);
    d.coef = cv.take<double>(6 * (size_t)E);
    d.Hpp = cv.take<double>(36 * (size_t)Np);
    d.Hll = cv.take<double>(9 * (size_t)L);
    d.b = cv.take<double>(nx);
    d.Dinv = cv.take<double>(9 * (size_t)L);
    d.S = cv.take<double>((size_t)n * n);
    d.x = cv.take<double>(nx);
    d.bs = cv.take<double>(n);
    d.red = cv.take<double>(8);
    d.flag = cv.take<int>(4);
    uint8_t* depth = cv.take<uint8_t>(E);
    if (n > 0) MAM_HIP(hipMemsetAsync(d.S, 0, sizeof(double) * (size_t)n * n, s));
    MAM_HIP(hipMemsetAsync(d.x, 0, sizeof(double) * nx, s));

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
        hipLaunchKernelGGL(mam::lba::k_reduce_chi, dim3(1), dim3(1024), 0, s, d, 0);
        MAM_HIP(hipMemcpyAsync(h_red, d.red, sizeof(double), hipMemcpyDeviceToHost, s));
        MAM_HIP(hipStreamSynchronize(s));
        *out_chi = h_red[0];
        return MAM_OK;
    };
    auto stopped = [&]() { return stop_flag && *stop_flag; };

    double chi0 = 0;
    if (int rc = chi_of(cur_pose, cur_pt, false, &chi0)) return rc;
    r->initial_chi2 = chi0;
    double currentLambda = -1.0, ni = 2.0;
    int nBad = 0, trials = 0, its = 0;
    bool ok = Np + L > 0;
    for (int it = 0; it < p->iterations && !stopped() && ok; it++) {
        double currentChi;
        {
            mam::StageTimer::Scope sc(&c->timer, s, 0);
            state(cur_pose, cur_pt, tr_pose, tr_pt);
            if (E > 0) hipLaunchKernelGGL(mam::lba::k_linearize, dim3(gE), dim3(256), 0, s, d, 1);
            hipLaunchKernelGGL(mam::lba::k_reduce_chi, dim3(1), dim3(1024), 0, s, d, 0);
            if (L > 0) hipLaunchKernelGGL(mam::lba::k_point_sys, dim3(gL), dim3(256), 0, s, d);
            if (Np > 0) hipLaunchKernelGGL(mam::lba::k_pose_sys, dim3(Np), dim3(64), 0, s, d);
            hipLaunchKernelGGL(mam::lba::k_max_diag, dim3(1), dim3(1024), 0, s, d);
        }
        MAM_HIP(hipMemcpyAsync(h_red, d.red, 3 * sizeof(double), hipMemcpyDeviceToHost, s));
        MAM_HIP(hipStreamSynchronize(s));
        currentChi = h_red[0];
        const double iniChi = currentChi;
        if (it == 0) { currentLambda = 1e-5 * h_red[2]; ni = 2; nBad = 0; }
        double rho = 0;
        int qmax = 0;
        do {
            {
                mam::StageTimer::Scope sc(&c->timer, s, 1);
                if (L > 0) hipLaunchKernelGGL(mam::lba::k_schur_prep, dim3(gL), dim3(256), 0, s, d, currentLambda);
                // the factorization leaves fill-in in S: clear the whole matrix before the blocks are rewritten
                if (n > 0) MAM_HIP(hipMemsetAsync(d.S, 0, sizeof(double) * (size_t)n * n, s));
                if (nbp > 0) hipLaunchKernelGGL(mam::lba::k_schur_blk, dim3(nbp), dim3(64), 0, s, d, currentLambda);
                if (Np > 0) hipLaunchKernelGGL(mam::lba::k_schur_rhs, dim3(Np), dim3(64), 0, s, d);
            }
            {
                mam::StageTimer::Scope sc(&c->timer, s, 2);
                MAM_HIP(hipMemsetAsync(d.flag, 0, sizeof(int), s));
                if (Np > 0) hipLaunchKernelGGL(mam::lba::k_ldlt, dim3(1), dim3(1024), 0, s, d);
            }
            {
                mam::StageTimer::Scope sc(&c->timer, s, 3);
                if (L > 0) hipLaunchKernelGGL(mam::lba::k_backsub, dim3(gL), dim3(256), 0, s, d);
                state(cur_pose, cur_pt, tr_pose, tr_pt);
                if (std::max(P, L) > 0) hipLaunchKernelGGL(mam::lba::k_update, dim3(gPL), dim3(256), 0, s, d);
                // chi2 of the trial state (errors kept: chi2() reads the last computeActiveErrors)
                state(tr_pose, tr_pt, tr_pose, tr_pt);
                if (E > 0) hipLaunchKernelGGL(mam::lba::k_linearize, dim3(gE), dim3(256), 0, s, d, 0);
                hipLaunchKernelGGL(mam::lba::k_reduce_chi, dim3(1), dim3(1024), 0, s, d, 0);
                hipLaunchKernelGGL(mam::lba::k_scale, dim3(1), dim3(1024), 0, s, d, currentLambda);
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
    double fchi = 0;
    if (int rc = chi_of(cur_pose, cur_pt, false, &fchi)) return rc;
    r->final_chi2 = fchi;
    r->iterations = its;
    r->lm_trials = trials;
    r->status = stopped() ? 1 : 0;
    return MAM_OK;
}

}  // extern "C"
