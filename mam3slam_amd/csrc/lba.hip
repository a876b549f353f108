// lba.hip — gfx950 Levenberg-Marquardt / Schur solve of Optimizer::LocalBundleAdjustment (include/mam_lba.h),
// batched over independent problems (one per agent / keyframe) with the LM control flow ON THE DEVICE.
//
// g2o semantics (BlockSolver_6_3 + LinearSolverEigen + OptimizationAlgorithmLevenberg, FP64) re-laid out for the
// GPU; every reduction has a fixed order so results are run-to-run reproducible:
//   k_linearize   per edge: map, error, chi2, Huber rho, Jacobians (OptimizableTypes.cpp:139-160), the robust-
//                 weighted terms constructQuadraticForm needs (base_binary_edge.hpp:75-112); chi2 partial sums
//   k_sys         per point: H_ll, b_l over its edge segment; one wave per non-fixed pose: H_pp, b_p
//   k_schur_prep  per point: D = H_ll + lambda I, D^-1, and per edge H_pl D^-1, H_pl D^-1 b_l (block_solver.hpp:
//                 405-427)
//   k_schur_blk   one wave per 6x6 block (i1 <= i2) of the reduced camera system, contributions in landmark
//                 order (block_solver.hpp:372-439), and b_s = b_p - sum of coefficients
//   k_ldlt        one workgroup per problem: blocked right-looking LDL^T of S (zero pivot = failure, as
//                 SimplicialLDLT), f64 MFMA trailing updates, fused forward / diagonal / backward substitution
//   k_backsub_update  x_l = D^-1 (b_l - H_pl^T x_p) (block_solver.hpp:461-482) and the trial state:
//                 T <- exp(dx) T (se3quat.h), X <- X + dx
//   k_ctl_end     on an iteration's first trial the iteration-start state first (levenberg.cpp:61-77, 171-185:
//                 chi2, lambda_0 = 1e-5 max diag(H) gathered by k_sys — the trial's kernels read lambda_0 through
//                 trial_lambda); then the trial's chi2, computeScale (partial sums from k_linearize), rho, accept (discardTop) /
//                 reject (pop), lambda update and the termination tests of levenberg.cpp:78-169 and
//                 sparse_optimizer.cpp:355-420
// Each kernel reads its problem's LM state (struct LM, device memory) and returns at once when the state says the
// stage is not due: the host enqueues whole "slots" (iteration start + one trial) for every problem of a batch and
// only synchronises once per chunk of slots (no host round trip per trial). Problems in different phases share the
// same launches.
#include <hip/hip_runtime.h>

#include <climits>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <numeric>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/mam_lba.h"
#include "camera.hpp"
#include "runtime.hpp"

namespace mam {
namespace lba {

// Levenberg state of one problem (levenberg.cpp members + the optimize() loop counters). The first 80 bytes are what
// kernels test and read on entry (LMHead: five 16-byte loads issued together, one memory round trip instead of a
// dependent load per field).
struct alignas(16) LM {
    int status;      // MAM_OK or MAM_ERR_*
    int done;        // optimize() returned
    int need_lin;    // the next slot starts an iteration (linearize + build)
    int cur;         // which state buffer holds the current estimate
    int fail;        // the last LDL^T hit a zero pivot
    int sys_ready;   // the iteration start's linearisation and system are built (the setup pass did iteration 0's)
    int tiles_lds;   // all non-zero tiles + y fit the factorization's LDS: k_ldlt_tiles factors in LDS
    int maxc;        // the most non-zero tiles below the diagonal tile in any block column (k_struct_tiles)
    int its, trials, qmax, nBad;
    int iterations;  // optimize(iterations)
    int ntiles;      // structurally non-zero 16x16 tiles of L (lower triangle incl. the diagonal; k_struct_tiles)
    int pad0, pad1;
    double lambda;
    unsigned long long maxdiag;   // max |diag(H)| of the iteration's system (bits of a non-negative double)
    double ni;
    double currentChi, iniChi, acceptedChi, initialChi;
    double scale_p;  // computeScale's pose part of the trial (the factorization's epilogue)
};
struct alignas(16) LMHead {
    int status, done, need_lin, cur, fail, sys_ready, tiles_lds, maxc, its, trials, qmax, nBad, iterations, ntiles,
        pad0, pad1;
    double lambda;
    unsigned long long maxdiag;
};
static_assert(sizeof(LMHead) == 80, "LMHead is the first 80 bytes of LM");
__device__ __forceinline__ LMHead lm_head(const LM* lm) {
    typedef __attribute__((address_space(1))) const int gi32;   // global loads (adjacent: merged into 16-byte loads)
    int v[20];
#pragma unroll
    for (int k = 0; k < 20; k++) v[k] = ((gi32*)lm)[k];
    LMHead h;
    __builtin_memcpy(&h, v, sizeof(h));
    return h;
}

// the column-chain factorization's per-problem ints: [0] claim counter, [1] the launch's base, [2] failure, [8 + k]
// column k's flag (k < 40), [48 + k] column k's ready flag
constexpr int MW_INTS = 96;   // (+ [48 + k] column k's ready flag: the lookahead form)

struct Prob {
    int P, L, E, Np, npad, n_cams, cam_model;
    double delta;                // Huber delta; <= 0: no robust kernel
    // inputs (point index = Hessian point index: points in ascending id order)
    const int32_t* edge_point;
    const int32_t* edge_pose;
    const double* edge_obs;
    const double* edge_w;        // invSigma2
    const uint8_t* active;       // [E] level-0 edges (NULL = all)
    const float* cams;           // [n_cams][4] pinhole or [n_cams][8] KB8
    const int32_t* pose_cam;     // NULL = camera 0
    const uint8_t* pose_fixed;
    const double* pose_q;        // [P][4] (input, device problems)
    const double* pose_t;        // [P][3]
    const double* point_xyz;     // [L][3]
    // structure
    int32_t* pose_h;             // Hessian pose block of pose (-1 fixed)
    int32_t* hpose;              // Hessian pose block -> pose
    int32_t* pe_off;             // per point: edge segment [pe_off[h], pe_off[h+1]) into pe_idx (edge order)
    int32_t* pe_idx;
    int32_t* slot_hp;            // per slot s of pe_idx: the Hessian pose block of edge pe_idx[s] (-1 fixed)
    int4* emeta;                 // per edge: (point, Hessian pose block or -1, first edge of its point, 0)
    int32_t* qe_off;             // per Hessian pose: edges (edge order)
    int32_t* qe_idx;
    int32_t* cnt;                // [L + Np] counters / cursors of the device structure build
    int32_t* eidx;               // [Np][L] edge of (pose block, point), never cleared: read through eidx_at
    uint8_t* pairmask;           // [Np][Np] (i1 < i2): the two poses share a landmark (S block non-zero)
    unsigned long long* pm_rows; // [64] (Np <= 64): pairmask row i1 as bits i2 (k_struct_sort; k_struct_tiles expands)
    int32_t* blk_off;            // [Np * Np + 1] start of block (i1, i2)'s landmark pairs in blk_pair (i1 <= i2); with
                                 // pair_fixed: the block's pair count, its pairs at the fixed offset i1 E + qe_off[i2]
    int pair_fixed;              // the pair buffer at its E Np bound: blocks at fixed offsets (no count / scan pass)
    int pw;                      // points per k_point_sys / k_point_trial workgroup of this batch (PW or PW_SMALL)
    int2* blk_pair;              // (edge of pose i1, edge of pose i2) per shared landmark, i2's edge order
    uint8_t* tmask;              // [nt][nt] (r >= c): 16x16 tile (r, c) of L is structurally non-zero (S + fill)
    int16_t* tslot;              // [nt][nt]: the tile's slot in the LDS tile pool (ldlt_tiles), -1 structurally zero
    int16_t* tlist;              // [ntiles][2]: (r, c) of each slot
    // per block column kc (nt <= 40, the LDS factorization): the rows r > kc of its non-zero tiles (clist, stride 40),
    // per block row kc the columns c < kc (rlist), their counts (ccnt[kc], ccnt[nt + kc]); k_struct_tiles
    int8_t* clist_g;
    int8_t* rlist_g;
    uint8_t* ccnt_g;
    // the order of S's pose blocks (k_struct_tiles): pose block h at position perm[h] (rows 6 perm[h] ..), iperm the
    // inverse; order_g: the block columns in the order the dataflow factorization takes them (by dependency level)
    int16_t* perm;
    int16_t* iperm;
    int8_t* order_g;
    double* pool;                // [ntiles][256]: S's non-zero tiles in slot order, each 16 x 16 tile as the LDS
                                 // factorization holds it (tsw layout); written by k_schur_blk when lm.tiles_lds
    int nt;                      // npad / 16
    // state: [2] buffers, lm->cur is the current one
    double* pose[2];             // [P][7] q(xyzw) t
    double* pt[2];               // [L][3]
    // per edge
    double* err;                 // [E][2]
    double* jac;                 // [E][21]: A(6) B(12) orr(2) wo(1)
    double* part_s;              // [ceil(E / 64) + 1] computeScale partial sums of k_linearize(trial)'s blocks
    double* part;                // [ceil(E / 256)] rho0 partial sums of k_linearize's blocks (trial, initial)
    double* part0;               // the same of k_linearize(iteration start), read by k_ctl_end's iteration-start step
    double* hpl;                 // [E][18] H_pl pose x landmark
    double* bdinv;               // [E][18] H_pl D^-1
    double* coef;                // [E][6]  H_pl D^-1 b_l
    // system
    double* Hpp;                 // [POSE_SPLIT][Np][36]: H_pp in partial sums (their fixed-order sum is the block)
    double* bp;                  // [POSE_SPLIT][Np][6]: b_p likewise (k_schur_blk sums them into b's pose part)
    double* Hll;                 // [L][9]
    double* b;                   // [6Np + 3L]
    double* Dinv;                // [L][9]
    double* S;                   // [npad][npad]
    double* x;                   // [6Np + 3L]
    double* bs;                  // [npad]
    double* ws;                  // LDL^T workspace when it does not fit in LDS (the column-chain form: y, D)
    int32_t* mw;                 // the column-chain form's claim counter, launch base, failure, column flags (MW_INTS)
    uint8_t* depth;              // [E] isDepthPositive of the final state
    LM* lm;
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

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

// fixed-order (butterfly) wave sum: every lane ends with the same value, deterministic run to run
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// The same butterfly sums for 4 Q values at once, reduce-scatter style: the xor-32 and xor-16 steps each exchange
// only the half of the values the lane keeps (a lane with the bit clear keeps the lower half), then the xor 8..1 steps
// on the Q values left. Lane group g = lane >> 4 ends with values [g Q, g Q + Q) — each one bit for bit what
// wave_sum_d returns for it (the same pairs added in the same order) — for 7 Q shuffles instead of 24 Q.
template <int Q>
__device__ __forceinline__ void wave_sum_scatter4(const double (&v)[4 * Q], double (&out)[Q]) {
    const int lane = lane_id();
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
}

// ---- per edge: error, robust weight, Jacobians (EdgeSE3ProjectXYZ); returns the edge's rho0
// jo / ho: where the edge's jac (21) and H_pl (18) records go (the caller's LDS staging slots); both are always
// written when want_jac (zeros where the edge is inactive or its pose fixed).
// linearize_edge_at: the same with the pose T and point X given (the fused point kernels hold X in LDS); write_err =
// false leaves d.err alone (a pass that only needs the Jacobian terms).
__device__ __forceinline__ double linearize_edge_at(const Prob& d, const double* T, const double* X, int ipose, int e,
                                                    bool want_jac, bool write_err, double* jo, double* ho) {
    double Xc[3];
    map_point(T, X, Xc);
    const bool kb8 = d.cam_model == MAM_CAM_KANNALA_BRANDT8;
    const float* c = d.cams + (kb8 ? 8 : 4) * (d.pose_cam ? d.pose_cam[ipose] : 0);
    double u, v;
    mam_camera cm;
    if (kb8) {
        cm.fx = c[0]; cm.fy = c[1]; cm.cx = c[2]; cm.cy = c[3];
        cm.k[0] = c[4]; cm.k[1] = c[5]; cm.k[2] = c[6]; cm.k[3] = c[7];
        cm.model = MAM_CAM_KANNALA_BRANDT8;
        cm.precision = 0.0f;
        cam::project_d(cm, Xc, &u, &v);   // KannalaBrandt8::project(Vector3d) (KannalaBrandt8.cpp:46-65)
    } else {
        u = c[0] * Xc[0] / Xc[2] + c[2];   // Pinhole::project (Pinhole.cpp:35-41)
        v = c[1] * Xc[1] / Xc[2] + c[3];
    }
    const double e0 = d.edge_obs[2 * e] - u, e1 = d.edge_obs[2 * e + 1] - v;
    if (write_err) {
        d.err[2 * e] = e0;
        d.err[2 * e + 1] = e1;
    }
    if (d.active && !d.active[e]) {
        // setLevel(1): outside initializeOptimization(0), no term in chi2 / H / b (zeros add exactly nothing)
        if (want_jac) {
            for (int k = 0; k < 21; k++) jo[k] = 0.0;
            for (int k = 0; k < 18; k++) ho[k] = 0.0;
        }
        return 0.0;
    }
    const double w = d.edge_w[e];
    const double chi = e0 * (w * e0) + e1 * (w * e1);
    double r0, r1;
    huber(chi, d.delta, &r0, &r1);
    if (!want_jac) return r0;
    const double x = Xc[0], y = Xc[1], z = Xc[2];
    // rotation matrix of T (Eigen toRotationMatrix)
    const double qx = T[0], qy = T[1], qz = T[2], qw = T[3];
    const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
    const double twx = tx * qw, twy = ty * qw, twz = tz * qw, txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz), tyz - twx,
                         txz - twy, tyz + twx, 1 - (txx + tyy)};
    double* o = jo;
    if (kb8) {
        // J = -projectJac(Xc) (KannalaBrandt8.cpp:145-175), A = J R, B = J * SE3deriv (OptimizableTypes.cpp:150-159)
        double P[6];
        cam::project_jac_d(cm, Xc, P);
        const double J[6] = {-P[0], -P[1], -P[2], -P[3], -P[4], -P[5]};
        for (int r = 0; r < 2; r++) {
            const double a0 = J[3 * r], a1 = J[3 * r + 1], a2 = J[3 * r + 2];
            for (int k = 0; k < 3; k++) o[3 * r + k] = a0 * R[k] + a1 * R[3 + k] + a2 * R[6 + k];
            double* B = o + 6 + 6 * r;
            // SE3deriv = [[0,z,-y,1,0,0],[-z,0,x,0,1,0],[y,-x,0,0,0,1]]
            B[0] = -a1 * z + a2 * y;
            B[1] = a0 * z - a2 * x;
            B[2] = -a0 * y + a1 * x;
            B[3] = a0;
            B[4] = a1;
            B[5] = a2;
        }
    } else {
        const double fx = c[0], fy = c[1];
        const double J0 = -(fx / z), J2 = -(-fx * x / (z * z)), J4 = -(fy / z), J5 = -(-fy * y / (z * z));
        // A = J R (2x3), J = [[J0, 0, J2], [0, J4, J5]]
        for (int k = 0; k < 3; k++) {
            o[k] = J0 * R[k] + J2 * R[6 + k];
            o[3 + k] = J4 * R[3 + k] + J5 * R[6 + k];
        }
        // B = J * SE3deriv, SE3deriv = [[0,z,-y,1,0,0],[-z,0,x,0,1,0],[y,-x,0,0,0,1]]
        o[6] = J2 * y;  o[7] = J0 * z - J2 * x; o[8] = -J0 * y; o[9] = J0; o[10] = 0.0; o[11] = J2;
        o[12] = -J4 * z + J5 * y; o[13] = -J5 * x; o[14] = J4 * x; o[15] = 0.0; o[16] = J4; o[17] = J5;
    }
    o[18] = -(w * e0) * r1;
    o[19] = -(w * e1) * r1;
    o[20] = r1 * w;
    // H_pl = B^T (rho' Omega) A for edges whose pose is optimised (base_binary_edge.hpp:54-120)
    if (d.pose_h[ipose] >= 0) {
        const double wo = r1 * w;
        for (int a = 0; a < 6; a++)
            for (int c2 = 0; c2 < 3; c2++) ho[3 * a + c2] = o[6 + a] * wo * o[c2] + o[12 + a] * wo * o[3 + c2];
    } else {
        for (int k = 0; k < 18; k++) ho[k] = 0.0;
    }
    return r0;
}

__device__ __forceinline__ double linearize_edge(const Prob& d, const double* pose, const double* pts, int e,
                                                 bool want_jac, double* jo, double* ho) {
    const int ip = d.edge_point[e], ipose = d.edge_pose[e];
    return linearize_edge_at(d, pose + 7 * (size_t)ipose, pts + 3 * (size_t)ip, ipose, e, want_jac, true, jo, ho);
}

// ================================================================================== device structure build
// The structure kernels run 256-thread workgroups: under the tracking load a 1024-thread workgroup waits for a CU
// with 16 free wave slots (their one-workgroup-per-problem scans took ~0.4 ms each beside tracking, µs alone).
constexpr int SB = 256;
// the pose x point table entry of (pose block h, point ip): the edge it holds when that edge really joins them, else
// -1 (the table is never cleared, so an entry left from an earlier problem in the arena is rejected here)
__device__ __forceinline__ int eidx_at(const Prob& d, const int32_t* row, int h, int ip) {
    const int e = row[ip];
    return ((unsigned)e < (unsigned)d.E && d.edge_point[e] == ip && d.pose_h[d.edge_pose[e]] == h) ? e : -1;
}

// For problems whose arrays are already in HBM (mam_lba_solve_batch_device): poses and points come in ascending id
// order (g2o's Hessian order, sparse_optimizer.cpp:166-190), so the pose blocks are a prefix count of the non-fixed
// poses and the point blocks are the identity; the per-point / per-pose edge lists (edge order) and the pose x point
// edge table are built here.

// grid (8, Q) x SB: block 0 scans pose_fixed -> pose_h / hpose; every block clears the counters, the pair mask
// and S's padding rows and seeds the state buffers (SE3Quat(q, t) normalises: w >= 0, unit). Neither the pose x point
// table nor the rest of S is cleared: a table entry is trusted only when it names an edge of that pose and point
// (eidx_at), and k_schur_blk writes every lower-triangle block of S each trial, the only part the factorization reads
// (its padding rows, below the identity block, stay the zeros written here). Under the tracking load these clears
// were ~1.4 MB per window of writes from workgroups waiting for CUs.
__global__ __launch_bounds__(SB) void k_struct_init(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    if (d.lm->status) return;
    const int t = threadIdx.x;
    const int gstride = gridDim.x * SB, g0 = blockIdx.x * SB + t;
    if (blockIdx.x == 0) {
        __shared__ int wsum[SB / 64];
        // pose_h: prefix count of non-fixed poses, SB per pass
        int base = 0;
        for (int c0 = 0; c0 < d.P; c0 += SB) {
            const int i = c0 + t;
            const int nf = (i < d.P && !d.pose_fixed[i]) ? 1 : 0;
            int v = nf;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int u = __shfl_up(v, o, 64);
                if (lane_id() >= o) v += u;
            }
            if (lane_id() == 63) wsum[t >> 6] = v;
            __syncthreads();
            int pre = 0, tot = 0;
            for (int w = 0; w < SB / 64; w++) {
                if (w < (t >> 6)) pre += wsum[w];
                tot += wsum[w];
            }
            if (i < d.P) {
                const int h = base + pre + v - nf;
                d.pose_h[i] = nf ? h : -1;
                if (nf) d.hpose[h] = i;
            }
            base += tot;
            __syncthreads();
        }
    }
    for (int i = g0; i < d.L + d.Np; i += gstride) d.cnt[i] = 0;
    if (g0 < MW_INTS) d.mw[g0] = 0;
    for (size_t i = g0; i < (size_t)d.Np * d.Np; i += gstride) d.pairmask[i] = 0;
    if (g0 < 64) d.pm_rows[g0] = 0ull;
    const size_t n6 = 6 * (size_t)d.Np;
    for (size_t i = g0; i < ((size_t)d.npad - n6) * d.npad; i += gstride) d.S[n6 * d.npad + i] = 0.0;
    for (int i = g0; i < d.P; i += gstride) {
        double q[4] = {d.pose_q[4 * i], d.pose_q[4 * i + 1], d.pose_q[4 * i + 2], d.pose_q[4 * i + 3]};
        if (q[3] < 0) for (int k = 0; k < 4; k++) q[k] = -q[k];
        const double nq = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (int k = 0; k < 4; k++) d.pose[0][7 * (size_t)i + k] = q[k] / nq;
        for (int k = 0; k < 3; k++) d.pose[0][7 * (size_t)i + 4 + k] = d.pose_t[3 * i + k];
    }
    for (int i = g0; i < 3 * d.L; i += gstride) d.pt[0][i] = d.point_xyz[i];
}

// grid (ceil(E/256), Q): per-point and per-pose edge counts; index validation. The pose counts go through a
// per-workgroup LDS histogram first (one device atomic per pose present in the workgroup instead of one per edge: a
// window's ~50 pose counters each took ~500 device atomics in turn, the contended part of the structure build)
constexpr int STRUCT_HIST = 512;   // poses the LDS histogram holds (larger windows: device atomics per edge)
__global__ __launch_bounds__(256) void k_struct_count(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    if (d.lm->status) return;
    __shared__ int hist[STRUCT_HIST];
    const bool lds_hist = d.Np <= STRUCT_HIST;
    if (lds_hist)
        for (int i = threadIdx.x; i < d.Np; i += 256) hist[i] = 0;
    __syncthreads();
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e < d.E) {
        const int ip = d.edge_point[e], ipose = d.edge_pose[e];
        if (ip < 0 || ip >= d.L || ipose < 0 || ipose >= d.P) {
            d.lm->status = MAM_ERR_ARG;
        } else {
            atomicAdd(&d.cnt[ip], 1);
            const int h = d.pose_h[ipose];
            if (h >= 0) {
                if (lds_hist) atomicAdd(&hist[h], 1);
                else atomicAdd(&d.cnt[d.L + h], 1);
            }
        }
    }
    __syncthreads();
    if (lds_hist)
        for (int i = threadIdx.x; i < d.Np; i += 256)
            if (hist[i]) atomicAdd(&d.cnt[d.L + i], hist[i]);
}

__device__ void block_excl_scan(const int32_t* in, int32_t* out, int n, int32_t* total_out) {
    __shared__ int wsum[SB / 64];
    __shared__ int carry;
    const int t = threadIdx.x;
    if (t == 0) carry = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += SB) {
        const int i = c0 + t;
        const int a = i < n ? in[i] : 0;
        int v = a;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(v, o, 64);
            if (lane_id() >= o) v += u;
        }
        if (lane_id() == 63) wsum[t >> 6] = v;
        __syncthreads();
        int pre = 0, tot = 0;
        for (int w = 0; w < SB / 64; w++) {
            if (w < (t >> 6)) pre += wsum[w];
            tot += wsum[w];
        }
        if (i < n) out[i] = carry + pre + v - a;
        __syncthreads();
        if (t == 0) carry += tot;
        __syncthreads();
    }
    if (t == 0) *total_out = carry;
}

// grid (1, Q) x SB: exclusive scans -> pe_off, qe_off; counters reset to be the scatter cursors
__global__ __launch_bounds__(SB) void k_struct_scan(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    if (d.lm->status) return;
    block_excl_scan(d.cnt, d.pe_off, d.L, d.pe_off + d.L);
    block_excl_scan(d.cnt + d.L, d.qe_off, d.Np, d.qe_off + d.Np);
    __syncthreads();
    for (int i = threadIdx.x; i < d.L + d.Np; i += SB) d.cnt[i] = 0;
}

// grid (ceil(E/256), Q): scatter into the lists (order fixed by k_struct_sort) and the pose x point table; a pose's
// slots for the workgroup's edges reserved by one device atomic (the LDS histogram's count), ranks from LDS atomics
__global__ __launch_bounds__(256) void k_struct_scatter(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    if (d.lm->status) return;
    __shared__ int hist[STRUCT_HIST];
    const bool lds_hist = d.Np <= STRUCT_HIST;
    if (lds_hist)
        for (int i = threadIdx.x; i < d.Np; i += 256) hist[i] = 0;
    __syncthreads();
    const int e = blockIdx.x * 256 + threadIdx.x;
    int h = -1, r = 0, ip = 0;
    if (e < d.E) {
        ip = d.edge_point[e];
        d.pe_idx[d.pe_off[ip] + atomicAdd(&d.cnt[ip], 1)] = e;
        h = d.pose_h[d.edge_pose[e]];
        if (h >= 0) {
            d.eidx[(size_t)h * d.L + ip] = e;
            if (lds_hist) r = atomicAdd(&hist[h], 1);
            else d.qe_idx[d.qe_off[h] + atomicAdd(&d.cnt[d.L + h], 1)] = e;
        }
    }
    if (!lds_hist) return;   // uniform
    __syncthreads();
    for (int i = threadIdx.x; i < d.Np; i += 256)
        if (hist[i]) hist[i] = atomicAdd(&d.cnt[d.L + i], hist[i]);   // the workgroup's base in pose i's list
    __syncthreads();
    if (h >= 0) d.qe_idx[d.qe_off[h] + hist[h] + r] = e;
}

// one point's edge list (n <= NR) sorted in registers (an unrolled exchange network; edge ids are distinct) with each
// dependent lookup issued for the whole list at once: three memory round trips instead of a few per element. The S
// blocks the landmark contributes to (g2o's BlockSolver keeps only these, block_solver.hpp:181-224) go to the LDS bit
// rows (rows != null: windows of <= 64 optimised poses) or straight to the byte pair mask.
template <int NR>
__device__ __forceinline__ void point_list_regs(const Prob& d, int h, int32_t* s, int n, unsigned long long* rows) {
    int v[NR], ep[NR], hv[NR];
#pragma unroll
    for (int a = 0; a < NR; a++) v[a] = a < n ? s[a] : INT_MAX;
    // (a list already in edge order — a window's edges listed point-major — skips the network)
    bool sorted = true;
#pragma unroll
    for (int a = 0; a + 1 < NR; a++) sorted = sorted && (a + 1 >= n || v[a] < v[a + 1]);
    if (!sorted)
#pragma unroll
        for (int i = 0; i < NR - 1; i++)
#pragma unroll
            for (int j = 0; j < NR - 1 - i; j++) {
                const int lo = min(v[j], v[j + 1]), hi = max(v[j], v[j + 1]);
                v[j] = lo;
                v[j + 1] = hi;
            }
#pragma unroll
    for (int a = 0; a < NR; a++) ep[a] = a < n ? d.edge_pose[v[a]] : 0;
#pragma unroll
    for (int a = 0; a < NR; a++) hv[a] = a < n ? d.pose_h[ep[a]] : -1;
#pragma unroll
    for (int a = 0; a < NR; a++)
        if (a < n) {
            s[a] = v[a];
            d.slot_hp[d.pe_off[h] + a] = hv[a];
            d.emeta[v[a]] = make_int4(h, hv[a], a == 0 ? 1 : 0, 0);
        }
    if (rows) {   // (bits mode: the point's pose mask; the workgroup folds the masks into the pair rows)
        unsigned long long m = 0;
#pragma unroll
        for (int a = 0; a < NR; a++) m |= hv[a] >= 0 ? 1ull << hv[a] : 0ull;
        *rows = m;
        return;
    }
#pragma unroll
    for (int a = 0; a < NR; a++)
#pragma unroll
        for (int b = a + 1; b < NR; b++) {
            const int ha = hv[a], hb = hv[b];
            if (ha >= 0 && hb >= 0 && hb != ha) d.pairmask[(size_t)min(ha, hb) * d.Np + max(ha, hb)] = 1;
        }
}

// grid (ceil(L/256) + Np, Q) x 256: restore edge order inside every list — per point its list sorted in registers (up
// to 32 observations; longer lists by one thread in place), per pose its segment ranked through a bitmap of the
// problem's edge ids (segments of up to 4096 edges in problems of up to 262144; else a bitonic sort in LDS, and
// longer segments, global BA, by odd-even transposition in place). Windows of <= 64
// optimised poses collect the pair mask as LDS bit rows per workgroup (one device atomic per row present instead of a
// byte store per observation pair: ~2.7M stores per batch of 32 ring windows), k_struct_tiles expands them.
#ifdef MAM_SORT_PROFILE
// cycles (thread 0, whole workgroup) of k_struct_sort's point workgroups [0] / pose workgroups [1], their counts [2] [3]
__device__ unsigned long long g_sortprof[4];
struct SortProf {
    long long t0 = clock64();
    int part;
    __device__ explicit SortProf(int p) : part(p) {}
    __device__ ~SortProf() {
        if (threadIdx.x == 0) {
            atomicAdd(&g_sortprof[part], (unsigned long long)(clock64() - t0));
            atomicAdd(&g_sortprof[2 + part], 1ull);
        }
    }
};
#endif
__global__ __launch_bounds__(256) void k_struct_sort(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    if (d.lm->status) return;
    const int nb_pts = (d.L + 255) / 256;
#ifdef MAM_SORT_PROFILE
    SortProf sp((int)blockIdx.x < nb_pts ? 0 : 1);
#endif
    if ((int)blockIdx.x < nb_pts) {
        // bits mode (Np <= 64): each thread leaves its point's pose mask in pm_s; row r of the pair mask is then the
        // OR over the masks holding r of their poses above r — one thread a row over the 256 masks (LDS broadcast
        // reads) instead of an LDS atomic per (point, pose): ~1.8k atomics on ~50 addresses a workgroup, ~100 us
        __shared__ unsigned long long pm_s[256];
        const bool bits = d.Np <= 64;   // uniform
        pm_s[threadIdx.x] = 0ull;
        unsigned long long* rows = bits ? pm_s + threadIdx.x : nullptr;
        const int h = blockIdx.x * 256 + threadIdx.x;
        if (h < d.L) {
            int32_t* s = d.pe_idx + d.pe_off[h];
            const int n = d.pe_off[h + 1] - d.pe_off[h];
            if (n <= 8) {
                point_list_regs<8>(d, h, s, n, rows);
            } else if (n <= 32) {
                point_list_regs<32>(d, h, s, n, rows);
            } else {
                // a long list (a ring window's MapPoints reach ~56 observations): 16 loads in flight a round (one
                // element a round trip took ~190 us for the window's longest lists); usually already in edge order,
                // sorted in place otherwise
                constexpr int CK = 16;
                bool sorted = true;
                for (int a0 = 0; a0 + 1 < n; a0 += CK) {
                    int w[CK + 1];
#pragma unroll
                    for (int u = 0; u <= CK; u++) w[u] = a0 + u < n ? s[a0 + u] : INT_MAX;
#pragma unroll
                    for (int u = 0; u < CK; u++) sorted = sorted && (a0 + u + 1 >= n || w[u] < w[u + 1]);
                }
                if (!sorted)
                    for (int k = 1; k < n; k++) {
                        const int v = s[k];
                        int m = k - 1;
                        while (m >= 0 && s[m] > v) { s[m + 1] = s[m]; m--; }
                        s[m + 1] = v;
                    }
                unsigned long long msk = 0;
                for (int a0 = 0; a0 < n; a0 += CK) {   // (the edges' pose blocks and metadata)
                    int ev[CK], pv[CK], hv2[CK];
#pragma unroll
                    for (int u = 0; u < CK; u++) ev[u] = a0 + u < n ? s[a0 + u] : 0;
#pragma unroll
                    for (int u = 0; u < CK; u++) pv[u] = a0 + u < n ? d.edge_pose[ev[u]] : 0;
#pragma unroll
                    for (int u = 0; u < CK; u++) hv2[u] = a0 + u < n ? d.pose_h[pv[u]] : -1;
#pragma unroll
                    for (int u = 0; u < CK; u++) {
                        if (a0 + u >= n) continue;
                        d.slot_hp[d.pe_off[h] + a0 + u] = hv2[u];
                        d.emeta[ev[u]] = make_int4(h, hv2[u], a0 + u == 0 ? 1 : 0, 0);
                        if (bits && hv2[u] >= 0) msk |= 1ull << hv2[u];
                    }
                }
                if (bits) {
                    *rows = msk;
                } else {
                    for (int a = 0; a < n; a++) {
                        const int ha = d.pose_h[d.edge_pose[s[a]]];
                        if (ha < 0) continue;
                        for (int b = a + 1; b < n; b++) {
                            const int hb = d.pose_h[d.edge_pose[s[b]]];
                            if (hb >= 0 && hb != ha) d.pairmask[(size_t)min(ha, hb) * d.Np + max(ha, hb)] = 1;
                        }
                    }
                }
            }
        }
        if (bits) {   // uniform
            __syncthreads();
            const int r = threadIdx.x;
            if (r < d.Np) {
                const unsigned long long above = ~((2ull << r) - 1ull);
                unsigned long long acc = 0ull;
                for (int i = 0; i < 256; i++) {
                    const unsigned long long m = pm_s[i];
                    if ((m >> r) & 1ull) acc |= m & above;
                }
                if (acc) atomicOr(&d.pm_rows[r], acc);
            }
        }
        return;
    }
    const int h = blockIdx.x - nb_pts;
    if (h >= d.Np) return;
    constexpr int CH = 4096;
    __shared__ int32_t seg[CH];
    int32_t* s = d.qe_idx + d.qe_off[h];
    const int n = d.qe_off[h + 1] - d.qe_off[h];
    constexpr int BMW = 8192;   // bitmap words: problems of <= 262144 edges
    if (n <= CH && d.E <= 32 * BMW) {
        // the segment's edge ids (distinct, in [0, E)) as a bitmap over the problem's edges; an id's rank = the set
        // bits before it: the per-thread word-range popcounts scanned once, then each id's rank from its own range.
        // Five barriers (the bitonic network's 66 stages of ~1.2k cycles each took ~37 us for a 1.7k-edge pose).
        __shared__ uint32_t bm[BMW];
        __shared__ int tpre[256], wsum2[4];
        const int t = threadIdx.x, nw = (d.E + 31) >> 5, per = (nw + 255) >> 8;
        for (int i = t; i < nw; i += 256) bm[i] = 0u;
        int ev[CH / 256];
#pragma unroll
        for (int u = 0; u < CH / 256; u++) ev[u] = t + 256 * u < n ? s[t + 256 * u] : -1;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < CH / 256; u++)
            if (ev[u] >= 0) atomicOr(&bm[ev[u] >> 5], 1u << (ev[u] & 31));
        __syncthreads();
        const int w0 = t * per, w1 = min(nw, w0 + per);
        int c = 0;
        for (int w = w0; w < w1; w++) c += __popc(bm[w]);
        int x = c;   // block exclusive scan of the per-thread counts
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if ((t & 63) >= o) x += y;
        }
        if ((t & 63) == 63) wsum2[t >> 6] = x;
        __syncthreads();
        int pre = x - c;
        for (int wv = 0; wv < (t >> 6); wv++) pre += wsum2[wv];
        tpre[t] = pre;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < CH / 256; u++) {
            const int e = ev[u];
            if (e < 0) continue;
            const int w = e >> 5, own = w / per;
            int r = tpre[own];
            for (int q = own * per; q < w; q++) r += __popc(bm[q]);
            r += __popc(bm[w] & ((1u << (e & 31)) - 1u));
            s[r] = e;
        }
    } else if (n <= CH) {
        // a bitonic sort of the segment padded to a power of two with INT_MAX (a rank count over the segment was
        // O(n^2): ~270 us per batch of 32 ring windows, ~1.7k edges per pose)
        int np2 = 1;
        while (np2 < n) np2 <<= 1;
        for (int i = threadIdx.x; i < np2; i += 256) seg[i] = i < n ? s[i] : INT_MAX;
        __syncthreads();
        for (int k = 2; k <= np2; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = threadIdx.x; t < (np2 >> 1); t += 256) {
                    const int i = 2 * t - (t & (j - 1)), l = i + j;   // pair (i, l = i + j), i with bit j clear
                    const int a = seg[i], b = seg[l];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        seg[i] = b;
                        seg[l] = a;
                    }
                }
                __syncthreads();
            }
        for (int i = threadIdx.x; i < n; i += 256) s[i] = seg[i];
    } else {
        // long segments (global BA): odd-even transposition in place, n rounds
        for (int round = 0; round < n; round++) {
            for (int i = 2 * threadIdx.x + (round & 1); i + 1 < n; i += 512) {
                const int a = s[i], b = s[i + 1];
                if (a > b) { s[i] = b; s[i + 1] = a; }
            }
            __syncthreads();
        }
    }
}

// ======================================================================================================= solve
// Per-edge records (jac 21 doubles, H_pl 18, W = H_pl D^-1 18, coefficients 6) are laid out edge-major; a wave owns 64
// consecutive edges and moves its records between HBM and LDS as contiguous 16-byte chunks (one cache line per 4
// lanes), the lanes computing on their own edge's record in LDS. (Per-lane strided 8-byte stores of a 168-byte record
// cost one L2 transaction per lane per store.)
constexpr int EW = 64;   // edges per wave
__device__ __forceinline__ void wave_copy_out(double* __restrict__ dst, const double* __restrict__ src, int n) {
    // n doubles from LDS to global, dst 16-byte aligned
    for (int i = 2 * lane_id(); i < n; i += 128) {
        if (i + 1 < n) *reinterpret_cast<double2*>(dst + i) = *reinterpret_cast<const double2*>(src + i);
        else dst[i] = src[i];
    }
}
__device__ __forceinline__ void wave_copy_in(double* __restrict__ dst, const double* __restrict__ src, int n) {
    for (int i = 2 * lane_id(); i < n; i += 128) {
        if (i + 1 < n) *reinterpret_cast<double2*>(dst + i) = *reinterpret_cast<const double2*>(src + i);
        else dst[i] = src[i];
    }
}

// The damping of this trial. On an iteration's first trial of the first iteration it is levenberg.cpp:71-77's
// lambda_0 = tau * max diag(H), tau = 1e-5 (computeLambdaInit :171-185), from the max k_sys gathered (max is exact in
// any order); k_ctl_end commits it to lm.lambda with the rest of the iteration-start state, so no control kernel runs
// between k_sys and the Schur kernels (one launch, and one dependency wait under load, fewer per trial).
__device__ __forceinline__ double trial_lambda(const LMHead& h) {
    return (h.need_lin && h.its == 0) ? 1e-5 * __longlong_as_double((long long)h.maxdiag) : h.lambda;
}
__device__ __forceinline__ double trial_lambda(const LM& lm) {
    return (lm.need_lin && lm.its == 0) ? 1e-5 * __longlong_as_double((long long)lm.maxdiag) : lm.lambda;
}

// grid (ceil(E/64), Q) x 64, the setup pass (once per solve): iteration 0's linearisation at the initial state — one
// wave per 64 edges: errors, Jacobians (jac, H_pl records, through one LDS staging buffer as contiguous 16-byte chunks)
// and the rho0 partial sum per wave (fixed-order butterfly) of the initial chi2. The trials' linearisations are the
// fused point kernels' (k_point_sys, k_point_trial).
__global__ __launch_bounds__(EW) void k_linearize(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    const LMHead hd = lm_head(d.lm);
    if (hd.status) return;
    __shared__ double sj[EW * 21];   // one staging buffer (LDS bounds the resident waves of this one-wave kernel)
    const int e0 = blockIdx.x * EW;
    if (e0 >= d.E) return;
    const int lane = lane_id(), e = e0 + lane;
    double jr[21], hr[18];   // the edge's records in registers, staged through one LDS buffer in turn
    double r = e < d.E ? linearize_edge(d, d.pose[hd.cur], d.pt[hd.cur], e, true, jr, hr) : 0.0;
    r = wave_sum_d(r);
    if (lane == 0) d.part0[blockIdx.x] = r;
    const int ne = min(EW, d.E - e0);
#pragma unroll
    for (int k = 0; k < 21; k++) sj[21 * lane + k] = jr[k];
    __syncthreads();
    wave_copy_out(d.jac + 21 * (size_t)e0, sj, 21 * ne);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 18; k++) sj[18 * lane + k] = hr[k];
    __syncthreads();
    wave_copy_out(d.hpl + 18 * (size_t)e0, sj, 18 * ne);
}

// grid (ceil(L/64) + Np, Q) x 64: H_ll, b_l per point (edge order, one thread each) and H_pp, b_p per optimised pose
// (one wave: lanes own strided edges, 27 register sums, fixed-order wave reduction)
// returns this thread's max |diag| of the blocks it wrote (0 for none; fmax drops NaN as the reference's max does)
#ifndef MAM_SYS_PF
#define MAM_SYS_PF 4
#endif
constexpr int SYS_PF = MAM_SYS_PF;   // edge indices per lane prefetched per pass (a pose: ~480 edges)
constexpr int PT_PF = 8;             // a point's edge indices prefetched per pass (a window's points: <= 8 edges)
// A pose's H_pp / b_p sums at an iteration start over POSE_SPLIT waves (slot chunks of 64 interleaved), each writing
// its partial sums; the consumers add the partials in part order. One wave per pose walked ~480 edges in 8 strides
// of dependent loads: the longest wave of k_point_sys.
#ifndef MAM_POSE_SPLIT
#define MAM_POSE_SPLIT 4
#endif
constexpr int POSE_SPLIT = MAM_POSE_SPLIT;
__device__ double sys_body(const Prob& d) {
    const int nb_pts = (d.L + 63) / 64;
    if ((int)blockIdx.x < nb_pts) {
        const int h = blockIdx.x * 64 + threadIdx.x;
        if (h >= d.L) return 0.0;
        double H[9] = {0}, bl[3] = {0};
        const int s1 = d.pe_off[h + 1];
        for (int sb = d.pe_off[h]; sb < s1; sb += PT_PF) {
            int pi[PT_PF];   // the point's edge indices loaded together, then their records in edge order
#pragma unroll
            for (int u = 0; u < PT_PF; u++) pi[u] = sb + u < s1 ? d.pe_idx[sb + u] : -1;
#pragma unroll
            for (int u = 0; u < PT_PF; u++) {
                if (pi[u] < 0) break;
                const double* j = d.jac + 21 * (size_t)pi[u];
                const double wo = j[20];
                for (int a = 0; a < 3; a++) {
                    bl[a] += j[a] * j[18] + j[3 + a] * j[19];
                    for (int c = 0; c < 3; c++) H[3 * a + c] += j[a] * wo * j[c] + j[3 + a] * wo * j[3 + c];
                }
            }
        }
        for (int k = 0; k < 9; k++) d.Hll[9 * (size_t)h + k] = H[k];
        for (int k = 0; k < 3; k++) d.b[6 * (size_t)d.Np + 3 * (size_t)h + k] = bl[k];
        return fmax(fmax(fabs(H[0]), fabs(H[4])), fabs(H[8]));
    }
    // POSE_SPLIT waves per pose, as the trials' pose_sys_wave: partial `part` sums the chunks part, part + POSE_SPLIT,
    // ... of 64 of the pose's edge list (a new keyframe's pose sees every MapPoint of its window: ~1.7k edges were 27
    // dependent strides of one wave); max |diag(H_pp)| over the summed partials in k_ctl_init
    const int hb = blockIdx.x - nb_pts, h = hb / POSE_SPLIT, part = hb % POSE_SPLIT, lane = threadIdx.x;
    if (h >= d.Np) return 0.0;
    double acc[27];
#pragma unroll
    for (int k = 0; k < 27; k++) acc[k] = 0.0;
    // the lane's edge indices of up to SYS_PF strides loaded together first (one memory round trip where there was
    // one per edge before its record's loads); the records then summed in the same order as before
    const int qs0 = d.qe_off[h], qs1 = d.qe_off[h + 1];
    for (int base = qs0 + 64 * part + lane; base < qs1; base += 64 * POSE_SPLIT * SYS_PF) {
        int qi[SYS_PF];
#pragma unroll
        for (int u = 0; u < SYS_PF; u++)
            qi[u] = base + 64 * POSE_SPLIT * u < qs1 ? d.qe_idx[base + 64 * POSE_SPLIT * u] : -1;
#pragma unroll
        for (int u = 0; u < SYS_PF; u++) {
            if (qi[u] < 0) break;
            const double* j = d.jac + 21 * (size_t)qi[u];
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
    }
    // 27 sums (+ one zero pad) reduce-scattered: lane group g holds sums [7 g, 7 g + 7), lane g * 16 + i sum 7 g + i
    double tot[7];
    {
        double v28[28];
#pragma unroll
        for (int k = 0; k < 27; k++) v28[k] = acc[k];
        v28[27] = 0.0;
        wave_sum_scatter4<7>(v28, tot);
    }
    const int g = lane >> 4, il = lane & 15;
    double val = 0.0;
#pragma unroll
    for (int i = 0; i < 7; i++) val = (il == i) ? tot[i] : val;
    const int q = 7 * g + il;   // this lane's sum (upper-triangle order of H, then b)
    if (il < 7 && q < 27) {
        if (q < 21) {
            int a = 0, r = q;
            while (r >= 6 - a) { r -= 6 - a; a++; }
            const int c = a + r;
            double* H = d.Hpp + 36 * ((size_t)part * d.Np + h);
            H[6 * a + c] = val;
            H[6 * c + a] = val;
        } else {
            d.bp[6 * ((size_t)part * d.Np + h) + (q - 21)] = val;   // (b's pose part: k_schur_blk sums the partials)
        }
    }
    return 0.0;
}

// Fixed-order sums over RED = 256 virtual threads (strided per-thread sums, then a tree), run by T real threads
// (T = 256, or 64 in a fused tail): thread t plays virtual threads t, t + T, ...; the same additions in the same
// order for every T, so a fused control step computes bit for bit what the one-workgroup kernel did.
constexpr int RED = 256;
template <int T>
__device__ double block_sum(const double* acc, double* s) {
#pragma unroll
    for (int v = 0; v < RED / T; v++) s[threadIdx.x + T * v] = acc[v];
    __syncthreads();
    for (int o = RED / 2; o > 0; o >>= 1) {
        for (int t = threadIdx.x; t < o; t += T) s[t] += s[t + o];
        __syncthreads();
    }
    const double r = s[0];
    __syncthreads();
    return r;
}

template <int T>
__device__ double chi_of_parts(const Prob& d, const double* part, double* s) {
    // parts of 64 edges, grouped by 256 as ((p0 + p1) + p2) + p3 (a missing part adds nothing), then strided + tree
    double acc[RED / T];
    const int np = (d.E + EW - 1) / EW, nb = (d.E + 255) / 256;
#pragma unroll
    for (int v = 0; v < RED / T; v++) {
        acc[v] = 0.0;
        for (int b = threadIdx.x + T * v; b < nb; b += RED) {
            double g = part[4 * b];
            for (int k = 1; k < 4; k++) g = g + (4 * b + k < np ? part[4 * b + k] : 0.0);
            acc[v] += g;
        }
    }
    return block_sum<T>(acc, s);
}

// grid (Q) x 256: the initial activeRobustChi2 (optimize() entry)
__global__ __launch_bounds__(RED) void k_ctl_init(const Prob* __restrict__ probs) {
    __shared__ double s[RED];
    const Prob& d = probs[blockIdx.x];
    LM& lm = *d.lm;
    if (lm.status) return;
    const double chi = chi_of_parts<RED>(d, d.part0, s);
    // max |diag(H_pp)| over the poses' summed POSE_SPLIT partials (k_sys' pose waves write partials; its point waves
    // already put max |diag(H_ll)| into lm.maxdiag), in k_schur_blk's summation order
    double pm = 0.0;
    for (int q = threadIdx.x; q < 6 * d.Np; q += RED) {
        const int h = q / 6, k = q % 6;
        double v = 0.0;
#pragma unroll
        for (int p = 0; p < POSE_SPLIT; p++) v += d.Hpp[36 * ((size_t)p * d.Np + h) + 7 * k];
        pm = fmax(pm, fabs(v));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pm = fmax(pm, __shfl_xor(pm, o));
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = pm;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 0; w < RED / 64; w++) pm = fmax(pm, s[w]);
        const double md = fmax(__longlong_as_double((long long)lm.maxdiag), pm);
        lm.maxdiag = (unsigned long long)__double_as_longlong(md);
        lm.initialChi = chi;
        lm.acceptedChi = chi;
        lm.currentChi = chi;
        lm.lambda = -1.0;
        lm.ni = 2.0;
        lm.its = lm.trials = lm.qmax = lm.nBad = 0;
        lm.fail = 0;
        lm.need_lin = 1;
        lm.sys_ready = 1;   // the setup's k_linearize + k_sys built iteration 0's system
        lm.done = (d.Np + d.L == 0 || lm.iterations <= 0) ? 1 : 0;
    }
}


// grid (ceil(L/64) + Np POSE_SPLIT, Q) x 64: the system (sys_body) and the points' max |diag(H_ll)| (one device atomic
// per wave; the poses' in k_ctl_init)
// (the setup pass: iteration 0's system; lambda_0 = 1e-5 max |diag(H)| is the only max the Levenberg loop reads)
__global__ __launch_bounds__(64) void k_sys(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    LM& lm = *d.lm;
    if (lm.status) return;
    double m = sys_body(d);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
    if (threadIdx.x == 0 && m > 0.0) atomicMax(&lm.maxdiag, (unsigned long long)__double_as_longlong(m));
}

// ---- Schur
// Entry (r, c) of a 16 x 16 tile in the LDS factorization's layout (column-major, rows XOR-swizzled by the column: the
// MFMA operand reads, the accumulator reads / writes and the row-per-thread panel rows are free of bank conflicts)
__host__ __device__ __forceinline__ int tsw(int r, int c) { return c * 16 + (r ^ c); }

// S(row, col) of the lower triangle: into the tile pool (problems factored in LDS: the tile's slot, skipped for a
// structurally zero tile, where only zeros land) or the dense npad x npad array
__device__ __forceinline__ void s_store(const Prob& d, bool pool, int row, int col, double v) {
    if (pool) {
        const int sl = d.tslot[(size_t)(row >> 4) * d.nt + (col >> 4)];
        if (sl >= 0) d.pool[(size_t)sl * 256 + tsw(row & 15, col & 15)] = v;
    } else {
        d.S[(size_t)row * d.npad + col] = v;
    }
}

// triangle index q -> (tr, tc), tc <= tr
__device__ __forceinline__ void tri_index(int q, int* tr, int* tc) {
    int r = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
    while (r * (r + 1) / 2 > q) r--;
    while ((r + 1) * (r + 2) / 2 <= q) r++;
    *tr = r;
    *tc = q - r * (r + 1) / 2;
}

// A short block's sum with one lane per entry of the 6x6 block (lanes 0..35 of one wave), each summing its entry over
// the block's landmark pairs in landmark order (g2o's order, block_solver.hpp:372-439): no reduction; 64 pair records
// fetched per coalesced load and broadcast by shuffles, 4 pairs' rows in flight per lane
__device__ __forceinline__ double schur_lane_sum(const Prob& d, int k0, int k1, int lane, bool act, int r36, int c36) {
    double acc = 0.0;
    const double* Wb = d.bdinv + 3 * r36;
    const double* Hb = d.hpl + 3 * c36;
    for (int kb = k0; kb < k1; kb += 64) {
        const int2 mine = kb + lane < k1 ? d.blk_pair[kb + lane] : make_int2(0, 0);
        const int n = min(64, k1 - kb);
        int j = 0;
        for (; j + 4 <= n; j += 4) {
            double w[4][3], b[4][3];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int px = __shfl(mine.x, j + u, 64), py = __shfl(mine.y, j + u, 64);
                if (act) {
#pragma unroll
                    for (int q = 0; q < 3; q++) {
                        w[u][q] = Wb[18 * (size_t)px + q];
                        b[u][q] = Hb[18 * (size_t)py + q];
                    }
                }
            }
            if (act) {
#pragma unroll
                for (int u = 0; u < 4; u++) acc += w[u][0] * b[u][0] + w[u][1] * b[u][1] + w[u][2] * b[u][2];
            }
        }
        for (; j < n; j++) {
            const int px = __shfl(mine.x, j, 64), py = __shfl(mine.y, j, 64);
            if (act)
                acc += Wb[18 * (size_t)px] * Hb[18 * (size_t)py] + Wb[18 * (size_t)px + 1] * Hb[18 * (size_t)py + 1] +
                       Wb[18 * (size_t)px + 2] * Hb[18 * (size_t)py + 2];
        }
    }
    return acc;
}

// grid (Np (Np + 1) / 2 + Np, Q) x SCHUR_T: one workgroup per block (i1 <= i2) of S (the triangle only: the upper
// half's workgroups would exit at once, half of the dispatches) over its landmark pairs (k_blk_fill): the waves take
// interleaved 64-pair chunks (a diagonal block has all ~480 of its pose's edges: one wave walked them in ~8 dependent
// strides), lanes strided over the pairs, a fixed-order wave sum, then the waves' partial sums added in wave order;
// then one workgroup per pose for b_s (and b's pose part: the sum of the POSE_SPLIT partials). Only the lower
// triangle of S is written (the one the factorization reads).
#ifndef MAM_SCHUR_PF
#define MAM_SCHUR_PF 2
#endif
constexpr int SCHUR_PF = MAM_SCHUR_PF;   // pair indices per lane prefetched per pass
#ifndef MAM_SCHUR_FULL
#define MAM_SCHUR_FULL 1   // a pair's two records loaded whole before its products (lone ring window 1.30 -> 1.26 ms; 0: in halves)
#endif
#ifndef MAM_SCHUR_T
#define MAM_SCHUR_T 128   // lone window: 64 / 128 / 256 threads 23.0 / 21.9 / 24.5 us per launch
#endif
#ifndef MAM_SCHUR_LANE_MAX
#define MAM_SCHUR_LANE_MAX 0   // blocks of at most this many landmark pairs: one wave, a lane per entry (0: never;
                               // 192 measured slower: ring batch 472 -> 603 us, world window 0.20 -> 0.32 ms per solve)
#endif
#ifndef MAM_SCHUR_T_BATCH
#define MAM_SCHUR_T_BATCH 64   // batches of >= 4 windows: 64 threads, records in halves (156 VGPRs: 3 waves a SIMD);
#endif                         // ring batch of 32: 14.34 -> 13.43 (64 threads) -> 13.20 ms (+ halves)
template <int SCHUR_T, bool FULL>
__global__ __launch_bounds__(SCHUR_T) void k_schur_blk(const Prob* __restrict__ probs) {
    constexpr int SCHUR_NW = SCHUR_T / 64;
    // XCD-aware: each XCD takes a contiguous range of (problem, block row) ids, so the W / H_pl records of the
    // landmarks its rows share stay in its L2
    const int lin = blockIdx.y * gridDim.x + blockIdx.x;
    const int logical = xcd_logical(lin, gridDim.x * gridDim.y);
    const int bt = logical % gridDim.x;
    const Prob& d = probs[logical / gridDim.x];
    const LM& lm = *d.lm;
    if (lm.status || lm.done) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int ntri = d.Np * (d.Np + 1) / 2;
    __shared__ double red[SCHUR_NW][36];
    if (bt >= ntri) {
        const int h = bt - ntri;
        if (h >= d.Np) return;
        double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        for (int s = d.qe_off[h] + threadIdx.x; s < d.qe_off[h + 1]; s += SCHUR_T) {
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
            red[wid][lane] = v;
        }
        __syncthreads();
        if (threadIdx.x < 6) {
            const int k = threadIdx.x;
            double v = 0.0, bsum = 0.0;
#pragma unroll
            for (int w = 0; w < SCHUR_NW; w++) v += red[w][k];
#pragma unroll
            for (int p = 0; p < POSE_SPLIT; p++) bsum += d.bp[6 * ((size_t)p * d.Np + h) + k];
            d.b[6 * (size_t)h + k] = bsum;
            d.bs[6 * (size_t)d.perm[h] + k] = bsum - v;   // (position order)
        }
        return;
    }
    // triangle row tr = the blocks of pose i1 = Np - 1 - tr (i2 = i1 .. Np - 1): a contiguous range of ids is a run
    // of i1 rows, the W records of pose i1's edges reused from the XCD's L2 as in the square grid
    int tr, tc;
    tri_index(bt, &tr, &tc);
    const int i1 = d.Np - 1 - tr, i2 = i1 + tc;
    const int bx = i1 * d.Np + i2;   // the block's pair-list slot
    // everything that depends only on the block index loaded at once (positions, pair mask, pair range, the diagonal
    // block's H_pp partials), then this thread's S entry's tile slot: two memory round trips before the pair records
    // instead of a chain of five
    const int p1 = d.perm[i1], p2 = d.perm[i2];
    const bool nz = i1 == i2 || d.pairmask[(size_t)i1 * d.Np + i2];
    const int k0 = d.pair_fixed ? i1 * d.E + d.qe_off[i2] : d.blk_off[bx];
    const int k1 = d.pair_fixed ? k0 + d.blk_off[bx] : d.blk_off[bx + 1];
    const bool pool = lm.tiles_lds != 0;
    const int q36 = threadIdx.x < 36 ? threadIdx.x : 0;
    double hs = 0.0;
    if (i1 == i2 && threadIdx.x < 36) {
#pragma unroll
        for (int p = 0; p < POSE_SPLIT; p++) hs += d.Hpp[36 * ((size_t)p * d.Np + i1) + q36];
    }
    // S(i1 row r, i2 col c) at the poses' positions, in the lower triangle
    const int r36 = q36 / 6, c36 = q36 % 6;
    const int srow = p2 >= p1 ? 6 * p2 + c36 : 6 * p1 + r36, scol = p2 >= p1 ? 6 * p1 + r36 : 6 * p2 + c36;
    const int sslot = (pool && threadIdx.x < 36) ? d.tslot[(size_t)(srow >> 4) * d.nt + (scol >> 4)] : -1;
    auto store = [&](double v) {
        if (pool) {
            if (sslot >= 0) d.pool[(size_t)sslot * 256 + tsw(srow & 15, scol & 15)] = v;
        } else {
            d.S[(size_t)srow * d.npad + scol] = v;
        }
    };
    if (!nz) {
        // no shared landmark: a zero block (the factorization's fill-in of the previous trial is overwritten)
        if (threadIdx.x < 36) store(0.0);
        return;
    }
    const double lambda = trial_lambda(lm);
    if (k1 - k0 <= MAM_SCHUR_LANE_MAX) {
        // a short block (most off-diagonal ones): the per-lane 36-entry sums would be mostly reduction
        if (wid != 0) return;
        const double v = schur_lane_sum(d, k0, k1, lane, threadIdx.x < 36, r36, c36);
        if (threadIdx.x < 36) {
            double out = -v;
            if (i1 == i2) out = (hs + (r36 == c36 ? lambda : 0.0)) - v;
            store(out);
        }
        return;
    }
    double acc[36];
#pragma unroll
    for (int k = 0; k < 36; k++) acc[k] = 0.0;
    for (int kb = k0 + 64 * wid + lane; kb < k1; kb += SCHUR_T * SCHUR_PF) {
        // the lane's pair records of up to SCHUR_PF strides loaded together (one round trip, not one per pair)
        int2 prs[SCHUR_PF];
#pragma unroll
        for (int u = 0; u < SCHUR_PF; u++) prs[u] = kb + SCHUR_T * u < k1 ? d.blk_pair[kb + SCHUR_T * u] : make_int2(-1, -1);
#pragma unroll
        for (int u = 0; u < SCHUR_PF; u++) {
            if (prs[u].x < 0) break;
            const int2 pr = prs[u];
            const double* W = d.bdinv + 18 * (size_t)pr.x;
            const double* B = d.hpl + 18 * (size_t)pr.y;
            if constexpr (FULL) {
            // both records loaded at once (9 16-byte loads each in flight together), then the products
            double wf[18], bf[18];
#pragma unroll
            for (int q = 0; q < 9; q++) {
                const double2 a = reinterpret_cast<const double2*>(W)[q], c = reinterpret_cast<const double2*>(B)[q];
                wf[2 * q] = a.x; wf[2 * q + 1] = a.y;
                bf[2 * q] = c.x; bf[2 * q + 1] = c.y;
            }
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int c = 0; c < 6; c++)
                    acc[6 * r + c] += wf[3 * r] * bf[3 * c] + wf[3 * r + 1] * bf[3 * c + 1] + wf[3 * r + 2] * bf[3 * c + 2];
            continue;
            }
            // rows of W and of H_pl three at a time (9 doubles each): no spill at 152 VGPRs; the same products summed
            // in the same order per accumulator
#pragma unroll
            for (int hr = 0; hr < 2; hr++) {
                double w[9];
#pragma unroll
                for (int q = 0; q < 9; q++) w[q] = W[9 * hr + q];
#pragma unroll
                for (int hc = 0; hc < 2; hc++) {
                    double b[9];
#pragma unroll
                    for (int q = 0; q < 9; q++) b[q] = B[9 * hc + q];
#pragma unroll
                    for (int r = 0; r < 3; r++)
#pragma unroll
                        for (int c = 0; c < 3; c++)
                            acc[6 * (3 * hr + r) + 3 * hc + c] +=
                                w[3 * r] * b[3 * c] + w[3 * r + 1] * b[3 * c + 1] + w[3 * r + 2] * b[3 * c + 2];
                }
            }
        }
    }
    // the 36 sums reduce-scattered per wave: lane group g holds sums [9 g, 9 g + 9); the waves' sums in wave order
    double tot[9];
    wave_sum_scatter4<9>(acc, tot);
    const int il = lane & 15, k = 9 * (lane >> 4) + il;
    if (il < 9) {
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < 9; i++) v = (il == i) ? tot[i] : v;
        red[wid][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < 36) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < SCHUR_NW; w++) v += red[w][q36];
        double out = -v;
        if (i1 == i2) out = (hs + (r36 == c36 ? lambda : 0.0)) - v;
        store(out);   // the lower triangle, the one the factorization reads
    }
}

// ---- dense LDL^T solve of S x = bs: one workgroup per problem, blocked right-looking, NB = 16 panels.
// S is npad x npad (npad = 6 Np rounded up to 16; the padding is an identity block after the real unknowns, so it
// changes nothing and every panel is full). Per panel:
//   (1) wave 0 factors the 16x16 diagonal block in registers: lane i owns row i, the pivot row is read with
//       a DPP broadcast within lanes 0..15, and solves the block of the forward substitution L11 y1 = y1;
//   (2) every thread takes one panel row: L21 = A21 L11^-T D^-1 (staged transposed in the panel workspace for the
//       trailing update) and the fused forward-substitution update y2 -= L21 y1;
//   (3) the trailing lower triangle A22 -= L21 D L21^T in 16x16 blocks, one wave each, as f64 MFMAs
//       (v_mfma_f64_16x16x4_f64) with both operands from the workspace; the next block column goes to an LDS
//       buffer that (1) and (2) of the next panel read.
// An exact zero pivot sets lm.fail (the failure rule of Eigen's SimplicialLDLT) and skips the solve.
// Then y /= D and the backward substitution L^T x = y, block by block, each thread updating its own y_i.
// The workspace (panel + y) is LDS when it fits (use_lds), else the problem's global scratch.
constexpr int NB = 16;
#ifndef MAM_LBA_ORDER
#define MAM_LBA_ORDER 1   // k_struct_tiles' two-chain pose order (0: the window's order)
#endif
constexpr int LDLT_TILES_NT_MAX = 40;   // ldlt_tiles' slot map in static LDS: nt <= 40 (npad <= 640)
#ifndef MAM_LDLT_THREADS
#define MAM_LDLT_THREADS 512
#endif
constexpr int LDLT_THREADS = MAM_LDLT_THREADS;

__host__ __device__ inline int ldlt_pad(int n) { return (n + NB - 1) / NB * NB; }

// ---- the landmark pairs of every S block, once per batch (the structure is fixed across the LM iterations):
// block (i1 <= i2) gets the (edge of pose i1, edge of pose i2) pairs of the landmarks both observe, in pose i2's
// edge order — k_schur_blk then walks only those instead of all of pose i2's edges through the pose x landmark table
__device__ __forceinline__ bool blk_nonzero(const Prob& d, int i1, int i2) {
    return i2 >= i1 && (i1 == i2 || d.pairmask[(size_t)i1 * d.Np + i2]);
}
// The pose-i1 edges of the landmarks pose i2's edges qe_idx[s0 + 64 u] observe (eidx_at for BLK_PF strides of the
// lane at once: each dependent lookup issued for the whole batch, five memory round trips per batch instead of per
// stride); ea[u] = -1 where there is none or past the list
constexpr int BLK_PF = 8;
__device__ __forceinline__ void blk_batch(const Prob& d, const int32_t* ei1, int i1, int s0, int end, int (&ec)[BLK_PF],
                                          int (&ea)[BLK_PF]) {
    int ip[BLK_PF], ep2[BLK_PF], eo[BLK_PF];
#pragma unroll
    for (int u = 0; u < BLK_PF; u++) ec[u] = s0 + 64 * u < end ? d.qe_idx[s0 + 64 * u] : -1;
#pragma unroll
    for (int u = 0; u < BLK_PF; u++) ip[u] = ec[u] >= 0 ? d.edge_point[ec[u]] : 0;
#pragma unroll
    for (int u = 0; u < BLK_PF; u++) {
        const int e = ec[u] >= 0 ? ei1[ip[u]] : -1;
        ea[u] = (unsigned)e < (unsigned)d.E ? e : -1;
    }
#pragma unroll
    for (int u = 0; u < BLK_PF; u++) {
        ep2[u] = ea[u] >= 0 ? d.edge_point[ea[u]] : -1;
        eo[u] = ea[u] >= 0 ? d.edge_pose[ea[u]] : 0;
    }
#pragma unroll
    for (int u = 0; u < BLK_PF; u++)
        if (ea[u] >= 0 && !(ep2[u] == ip[u] && d.pose_h[eo[u]] == i1)) ea[u] = -1;
}
// grid (Np * Np, Q) x 64: pairs per block
__global__ __launch_bounds__(64) void k_blk_count(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    if (d.lm->status) return;
    const int bx = blockIdx.x;
    if (bx >= d.Np * d.Np) return;
    const int i1 = bx / d.Np, i2 = bx % d.Np, lane = threadIdx.x;
    int n = 0;
    if (blk_nonzero(d, i1, i2)) {
        const int32_t* ei1 = d.eidx + (size_t)i1 * d.L;
        const int end = d.qe_off[i2 + 1];
        for (int s0 = d.qe_off[i2] + lane; s0 < end; s0 += 64 * BLK_PF) {
            int ec[BLK_PF], ea[BLK_PF];
            blk_batch(d, ei1, i1, s0, end, ec, ea);
#pragma unroll
            for (int u = 0; u < BLK_PF; u++) n += ea[u] >= 0;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
    }
    if (lane == 0) d.blk_off[bx] = n;
}
// grid (1, Q) x SB: exclusive scan of the counts, the total at [Np * Np]
__global__ __launch_bounds__(SB) void k_blk_scan(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    if (d.lm->status) return;
    __shared__ int part[SB];
    const int n = d.Np * d.Np, t = threadIdx.x;
    const int per = (n + SB - 1) / SB, b = t * per, e = min(n, b + per);
    int sum = 0;
    for (int i = b; i < e; i++) sum += d.blk_off[i];
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < SB; o <<= 1) {   // inclusive Hillis-Steele
        const int v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = t > 0 ? part[t - 1] : 0;
    for (int i = b; i < e; i++) {
        const int c = d.blk_off[i];
        d.blk_off[i] = run;
        run += c;
    }
    if (t == SB - 1) d.blk_off[n] = part[SB - 1];
}
// grid (Np * Np, Q) x 64: the pairs, compacted in edge order by ballot
__global__ __launch_bounds__(64) void k_blk_fill(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    if (d.lm->status) return;
    const int bx = blockIdx.x;
    if (bx >= d.Np * d.Np) return;
    const int i1 = bx / d.Np, i2 = bx % d.Np, lane = threadIdx.x;
    if (!blk_nonzero(d, i1, i2)) {
        if (d.pair_fixed && lane == 0) d.blk_off[bx] = 0;
        return;
    }
    const int32_t* ei1 = d.eidx + (size_t)i1 * d.L;
    // pair_fixed: the block's pairs at i1 E + qe_off[i2] (at most pose i2's edge count: the E Np buffer holds every
    // block without a count pass), its count left in blk_off[bx]
    const int base0 = d.pair_fixed ? i1 * d.E + d.qe_off[i2] : d.blk_off[bx];
    int base = base0;
    const int end = d.qe_off[i2 + 1];
    // (every lane runs the batches of the longest lane: the ballots need the whole wave)
    for (int c0 = d.qe_off[i2]; c0 < end; c0 += 64 * BLK_PF) {
        int ec[BLK_PF], ea[BLK_PF];
        blk_batch(d, ei1, i1, c0 + lane, end, ec, ea);
#pragma unroll
        for (int u = 0; u < BLK_PF; u++) {   // the 64-slot chunks in list order
            const bool hit = ea[u] >= 0;
            const uint64_t m = __ballot(hit);
            if (hit) d.blk_pair[base + __popcll(m & ((1ull << lane) - 1ull))] = make_int2(ea[u], ec[u]);
            base += __popcll(m);
        }
    }
    if (d.pair_fixed && lane == 0) d.blk_off[bx] = base - base0;
}

// grid (Q) x SB, after k_struct_sort: the 16x16 tile pattern of L. A tile of S is non-zero when it holds a pose
// diagonal block or the block of two poses sharing a landmark (pairmask); the right-looking factorization then fills
// tile (r1, r2) whenever tiles (r1, c) and (r2, c) are non-zero for some c < r2 (the symbolic LDL^T at tile
// granularity, column by column — what SimplicialLDLT's symbolic phase does per entry, linear_solver_eigen.h:147-201).
// Structurally zero tiles of L stay exact zeros, so k_ldlt skips them: every non-zero entry sees the same arithmetic
// as in the dense factorization. Windows whose covisibility is banded (keyframes along a trajectory) factor in
// O(n b^2) instead of O(n^3).
__global__ __launch_bounds__(SB) void k_struct_tiles(const Prob* __restrict__ probs, int lds_bytes) {
    const Prob& d = probs[blockIdx.x];
    if (d.lm->status) return;
    const int nt = d.nt, n = 6 * d.Np, Np = d.Np;
    const int t = threadIdx.x, lane = t & 63;
    // Windows of up to 64 tiles and 128 poses (every window the LDS factorization takes) work on LDS copies of the
    // pair mask and the tile mask, and run the symbolic factorization and the dependency levels in one wave on 64-bit
    // tile rows (lane r: row r of L's tile pattern) — the global-memory form below walks the same steps with a barrier
    // per block column.
    const bool small = nt <= 64 && Np <= 128;
    __shared__ uint8_t pm_s[128 * 128];
    __shared__ uint8_t tm_s[64 * 64];
    __shared__ int16_t ip_s[128];
    __shared__ int bw, nnz;
    const uint8_t* pm = small ? pm_s : d.pairmask;
    uint8_t* tm = small ? tm_s : d.tmask;
    const int16_t* ip = small ? ip_s : d.iperm;
    if (t == 0) bw = 0;
    if (Np <= 64) {
        // k_struct_sort's bit rows expanded into the byte mask (the LDS copy here, the global one for k_blk_* and
        // k_schur_blk)
        for (int q = t; q < Np * Np; q += SB) {
            const int i1 = q / Np, i2 = q % Np;
            const uint8_t v = (uint8_t)((d.pm_rows[i1] >> i2) & 1ull);
            pm_s[q] = v;
            d.pairmask[q] = v;
        }
    } else if (small) {
        for (int q = t; q < Np * Np; q += SB) pm_s[q] = d.pairmask[q];
    }
    __syncthreads();
    // The pose order. For a banded pose graph (bandwidth b: poses more than b apart in the window share no landmark),
    // [0, m) | [m + s, Np) reversed | [m, m + s), s >= b: no S entry couples the two ends, so they factor as two
    // independent dependency chains of about half the length and the separator follows (nested dissection, one
    // level; Eigen's SimplicialLDLT orders with AMD for the same reason: linear_solver_eigen.h). m and m + (Np - m - s)
    // are multiples of 8 poses (48 rows: three tiles), so no 16-row tile holds poses of two parts. Kept only when the
    // reordered pattern (its fill included) still fits the LDS factorization; otherwise the window's own order.
    {
        int lb = 0;
        for (int q = t; q < Np * Np; q += SB) {
            const int i1 = q / Np, i2 = q % Np;
            if (i2 > i1 && pm[q]) lb = max(lb, i2 - i1);
        }
        for (int o = 32; o > 0; o >>= 1) lb = max(lb, __shfl_xor(lb, o, 64));
        if (lane == 0 && lb > 0) atomicMax(&bw, lb);
    }
    __syncthreads();
    const int b = bw;
    int sep = b;
    while ((Np - sep) % 8) sep++;
    const int m = (Np - sep) / 16 * 8, nb = Np - sep - m;
    for (int attempt = MAM_LBA_ORDER && b > 0 && m >= 8 && nb >= 8 ? 0 : 1; attempt < 2; attempt++) {
        for (int h = t; h < Np; h += SB) {
            int p = h;
            if (attempt == 0) p = h >= m + sep ? m + (Np - 1 - h) : h >= m ? h + nb : h;
            d.perm[h] = (int16_t)p;
            d.iperm[p] = (int16_t)h;
            if (small) ip_s[p] = (int16_t)h;
        }
        if (t == 0) nnz = 0;
        __syncthreads();
        for (int q = t; q < nt * nt; q += SB) {
            const int r = q / nt, c = q % nt;
            uint8_t v = 0;
            if (r == c) {
                v = 1;
            } else if (r > c) {
                const int r0 = NB * r, r1 = min(NB * r + NB, n), c0 = NB * c, c1 = min(NB * c + NB, n);
                if (r0 < r1 && c0 < c1) {
                    for (int p1 = c0 / 6; p1 <= (c1 - 1) / 6 && !v; p1++)
                        for (int p2 = r0 / 6; p2 <= (r1 - 1) / 6 && !v; p2++) {
                            const int i1 = ip[p1], i2 = ip[p2];
                            if (i1 == i2 || pm[(size_t)min(i1, i2) * Np + max(i1, i2)]) v = 1;
                        }
                }
            }
            tm[q] = v;
        }
        __syncthreads();
        if (small) {
            // the right-looking symbolic LDL^T at tile granularity: column c's pattern is final once the columns before
            // it are done; every row r1 > c holding tile (r1, c) fills (r1, r2) for the rows c < r2 <= r1 of column c
            if (t < 64) {
                uint64_t R = 0;
                if (lane < nt)
                    for (int c = 0; c <= lane; c++) R |= (uint64_t)(tm_s[lane * nt + c] != 0) << c;
                for (int c = 0; c + 1 < nt; c++) {
                    const uint64_t col = __ballot(((R >> c) & 1) != 0);
                    if (lane > c && ((R >> c) & 1)) {
                        const uint64_t upto = lane >= 63 ? ~0ull : ((2ull << lane) - 1);
                        R |= col & upto & ~((2ull << c) - 1);
                    }
                }
                int cnt = 0;
                if (lane < nt) {
                    for (int c = 0; c < nt; c++) tm_s[lane * nt + c] = (uint8_t)((R >> c) & 1);
                    cnt = __popcll(R);
                }
                for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
                if (lane == 0) nnz = cnt;
            }
        } else {
            for (int c = 0; c + 1 < nt; c++) {
                const int mm = nt - 1 - c;
                for (int q = t; q < mm * mm; q += SB) {
                    const int r1 = c + 1 + q / mm, r2 = c + 1 + q % mm;
                    if (r2 <= r1 && tm[(size_t)r1 * nt + c] && tm[(size_t)r2 * nt + c]) tm[(size_t)r1 * nt + r2] = 1;
                }
                __syncthreads();
            }
            int cnt = 0;
            for (int q = t; q < nt * nt; q += SB) cnt += tm[q];
            atomicAdd(&nnz, cnt);
        }
        __syncthreads();
        if (attempt == 0 && nt <= LDLT_TILES_NT_MAX &&
            (size_t)nnz * 256 * sizeof(double) + (size_t)d.npad * sizeof(double) <= (size_t)lds_bytes)
            break;   // uniform
        __syncthreads();
    }
    if (small)
        for (int q = t; q < nt * nt; q += SB) d.tmask[q] = tm_s[q];
    // the non-zero tiles' slots in ldlt_tiles' LDS pool (row-major order of (r, c), r >= c), their count, and whether
    // the pool and y fit the factorization's dynamic LDS (lds_bytes)
    __shared__ int wsum[SB / 64];
    __shared__ int carry;
    __shared__ int16_t sl_last[64];   // the last tile row's slots (the padding loop below reads them from LDS)
    if (t == 0) carry = 0;
    __syncthreads();
    for (int c0 = 0; c0 < nt * nt; c0 += SB) {
        const int q = c0 + t;
        const int f = (q < nt * nt && tm[q]) ? 1 : 0;
        int v = f;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(v, o, 64);
            if (lane_id() >= o) v += u;
        }
        if (lane_id() == 63) wsum[t >> 6] = v;
        __syncthreads();
        int pre = 0, tot = 0;
        for (int w = 0; w < SB / 64; w++) {
            if (w < (t >> 6)) pre += wsum[w];
            tot += wsum[w];
        }
        if (q < nt * nt) {
            const int sl = carry + pre + v - f;
            d.tslot[q] = f ? (int16_t)sl : (int16_t)-1;
            if (f) {
                d.tlist[2 * sl] = (int16_t)(q / nt);
                d.tlist[2 * sl + 1] = (int16_t)(q % nt);
            }
            if (q / nt == nt - 1 && q % nt < 64) sl_last[q % nt] = f ? (int16_t)sl : (int16_t)-1;
        }
        __syncthreads();
        if (t == 0) carry += tot;
        __syncthreads();
    }
    if (t == 0) {
        LM& lm = *d.lm;
        lm.ntiles = carry;
        lm.tiles_lds = (nt <= LDLT_TILES_NT_MAX && (size_t)carry * 256 * sizeof(double) + (size_t)d.npad * sizeof(double) <=
                                                        (size_t)lds_bytes) ? 1 : 0;
    }
    __syncthreads();
    // the factorization's column / row lists (what it walked its slot map for at every launch), and the pool's padding
    // rows (the last tile row, rows >= n: an identity block after the unknowns, zeros elsewhere; k_schur_blk writes
    // every other entry of the pool every trial)
    __shared__ int maxc;
    if (t == 0) maxc = 0;
    __syncthreads();
    if (nt <= LDLT_TILES_NT_MAX) {
        for (int k = t; k < nt; k += SB) {
            int nc = 0, nr = 0;
            for (int r = k + 1; r < nt; r++)
                if (tm[(size_t)r * nt + k]) d.clist_g[k * 40 + nc++] = (int8_t)r;
            for (int c = 0; c < k; c++)
                if (tm[(size_t)k * nt + c]) d.rlist_g[k * 40 + nr++] = (int8_t)c;
            d.ccnt_g[k] = (uint8_t)nc;
            d.ccnt_g[nt + k] = (uint8_t)nr;
            atomicMax(&maxc, nc);
        }
        // the dataflow order: block columns by dependency level (1 + the deepest column they pull from), then index —
        // with the split pose order the two ends' columns alternate. One wave, lane k: column k's parents (the
        // columns c < k of row k's non-zero tiles) as a bit row; level l = the columns whose parents all have levels
        // < l (Kahn's layering: the longest dependency path), positions by a prefix count within the level.
        if (t < 64) {
            uint64_t P = 0;
            if (lane < nt)
                for (int c = 0; c < lane; c++) P |= (uint64_t)(tm[(size_t)lane * nt + c] != 0) << c;
            const uint64_t all = nt >= 64 ? ~0ull : ((1ull << nt) - 1);
            uint64_t done = 0;
            int base = 0;
            for (int l = 0; done != all && l < 64; l++) {
                const uint64_t ready = __ballot(lane < nt && !((done >> lane) & 1) && (P & ~done) == 0);
                if ((ready >> lane) & 1) d.order_g[base + __popcll(ready & ((1ull << lane) - 1))] = (int8_t)lane;
                base += __popcll(ready);
                done |= ready;
            }
        }
        if (nt > 0)
            for (int q = t; q < nt * 256; q += SB) {
                const int c = q >> 8, e = q & 255;
                const int j = e >> 4, i = (e & 15) ^ j;   // tsw(i, j) = j * 16 + (i ^ j)
                const int gi = NB * (nt - 1) + i, gj = NB * c + j;
                const int sl = sl_last[c];   // (nt <= LDLT_TILES_NT_MAX < 64)
                if (gi >= n && sl >= 0) d.pool[(size_t)sl * 256 + e] = gi == gj ? 1.0 : 0.0;
            }
    }
    __syncthreads();
    if (t == 0) d.lm->maxc = maxc;
}


// workspace doubles: the panel PL (NB x (npad - NB), L21 transposed), the block column CB (NB x (npad + 1),
// column-major with an odd stride) and y (npad)
__host__ __device__ inline int ldlt_cb_stride(int npad) { return npad + 1; }
__host__ __device__ inline size_t ldlt_ws_doubles(int npad) {
    const int m = npad > NB ? npad - NB : 0;
    return (size_t)NB * (size_t)m + (size_t)NB * (size_t)ldlt_cb_stride(npad) + (size_t)npad;
}
__host__ __device__ inline size_t ldlt_lds_bytes(int npad) { return ldlt_ws_doubles(npad) * sizeof(double); }

// S in the global address space: flat accesses would count in lgkmcnt too, so every LDS wait would also wait for the
// A loads in flight (the prefetches across the panel rows)
typedef __attribute__((address_space(1))) double gdouble;
// lane k of each 16-lane row, in every lane of that row (DPP row_newbcast: a VGPR result, no SGPR round trip and none
// of v_readlane's hazards); k a constant after unrolling
__device__ __forceinline__ int bcast16_i(int v, int k) {
    switch (k) {
#define MAM_BC(n) \
    case n: return __builtin_amdgcn_mov_dpp(v, 0x150 + n, 0xf, 0xf, false);
        MAM_BC(0) MAM_BC(1) MAM_BC(2) MAM_BC(3) MAM_BC(4) MAM_BC(5) MAM_BC(6) MAM_BC(7)
        MAM_BC(8) MAM_BC(9) MAM_BC(10) MAM_BC(11) MAM_BC(12) MAM_BC(13) MAM_BC(14) MAM_BC(15)
#undef MAM_BC
    }
    return 0;
}
// the double form: one v_mov_b64_dpp (gfx950 DPP64 supports row_newbcast) instead of two 32-bit moves
__device__ __forceinline__ double bcast16_d(double v, int k) {
    switch (k) {
#define MAM_BC(n) \
    case n: return __builtin_amdgcn_mov_dpp(v, 0x150 + n, 0xf, 0xf, false);
        MAM_BC(0) MAM_BC(1) MAM_BC(2) MAM_BC(3) MAM_BC(4) MAM_BC(5) MAM_BC(6) MAM_BC(7)
        MAM_BC(8) MAM_BC(9) MAM_BC(10) MAM_BC(11) MAM_BC(12) MAM_BC(13) MAM_BC(14) MAM_BC(15)
#undef MAM_BC
    }
    return 0.0;
}

// acc += (value of src in lane K of this lane's 16-lane row) * m: the broadcast folded into the FMA as one
// v_fmac_f64_dpp row_newbcast (gfx950 DPP64); one instruction where a v_mov_b64_dpp + v_fma_f64 pair was. The s_nop
// covers the VALU-write -> DPP-read hazard on src (inline asm is not seen by the hazard recognizer); not volatile, so
// the scheduler may interleave independent work. Same rounding as fma(src_K, m, acc).
// NOP = false where src was last written many instructions earlier (the later FMAs of one step).
template <int K, bool NOP = true>
__device__ __forceinline__ void fmac_bcast16(double& acc, double src, double m) {
    if constexpr (NOP)
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
            : "+v"(acc)
            : "v"(src), "v"(m), "n"(K));
    else
        asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
            : "+v"(acc)
            : "v"(src), "v"(m), "n"(K));
}
template <int J, int K>
struct Fmac16 {
    // step J's FMAs all read src = A(., J) (written by step J - 1's first FMA, at least a step earlier); the first
    // keeps the hazard nop, the DPP reads after it are two or more instructions past any write of src
    __device__ __forceinline__ static void run(double* row, double a, double ml) {
        fmac_bcast16<K, K == J + 1>(row[K], a, ml);
        Fmac16<J, K + 1>::run(row, a, ml);
    }
};
template <int J>
struct Fmac16<J, NB> {
    __device__ __forceinline__ static void run(double*, double, double) {}
};
template <int J>
struct Diag16 {
    // step J of the right-looking LDL^T of the lanes' rows: A(lane, k) -= l(lane, J) A(k, J), k > J, with
    // l(lane, J) = A(lane, J) / d_J; A(k, J) is the pre-scaling column, broadcast from lane k, so the update does not
    // wait for the pivot's reciprocal
    __device__ __forceinline__ static void run(double* row, double& dmine, int lane) {
        const double a = row[J];
        const double dj = bcast16_d(a, J);
        if (lane == J) dmine = dj;
        // the pivot's reciprocal by v_rcp_f64 and two Newton steps (within an ulp of 1/dj; the divide's scale /
        // fixup steps guard denormal and huge pivots, which a damped system's diagonal does not have) — it is the
        // serial part of every step
        double inv = __builtin_amdgcn_rcp(dj);
        inv = fma(inv, fma(-dj, inv, 1.0), inv);
        inv = fma(inv, fma(-dj, inv, 1.0), inv);
        if (dj == 0.0) inv = 0.0;
        const double l = a * inv;
        Fmac16<J, J + 1>::run(row, a, -l);
        if (lane > J) row[J] = l;
        Diag16<J + 1>::run(row, dmine, lane);
    }
};
template <>
struct Diag16<NB> {
    __device__ __forceinline__ static void run(double*, double&, int) {}
};

// wave-level LDL^T of a 16x16 block held one row per lane (lanes 0..15; the other lanes carry zeros): on entry
// row[c] = A(lane, c) (c <= lane read), on exit row[c] = L(lane, c) for c < lane and D(lane) at c == lane (the entries
// above the diagonal are don't-care values nothing reads); returns D(lane)
__device__ __forceinline__ double diag16_factor(double row[NB], int lane) {
    double dmine = 1.0;
    Diag16<0>::run(row, dmine, lane);
    return dmine;
}

// the forward block solve y1 <- L11^-1 y1 on the factored rows (lane i: y_i)
__device__ __forceinline__ double diag16_forward(const double row[NB], double yv, int lane) {
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const double yj = bcast16_d(yv, j);
        if (lane > j) yv = fma(-row[j], yj, yv);
    }
    return yv;
}

// wave 0: LDL^T of the 16x16 diagonal block at kb, read from the block-column buffer (CB[c * cs + r] = A(kb + r,
// kb + c), final), written back to A (L below, D on the diagonal), plus Ld (L11, row-major), dk / invdk (D and 1/D)
// for the panel rows and the trailing update, and the forward block solve of y.
__device__ __forceinline__ void ldlt_diag(gdouble* A, int N, int kb, const double* CB, int cs, double* Y, double* Ld,
                                          double* dk, double* invdk, int* fail, int lane) {
    double row[NB];
#pragma unroll
    for (int c = 0; c < NB; c++) row[c] = lane < NB ? CB[(size_t)c * cs + lane] : 0.0;
    const double dmine = diag16_factor(row, lane);
    const double yv = diag16_forward(row, lane < NB ? Y[kb + lane] : 0.0, lane);
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

// One wave: NT 16x16 blocks (br[t], bc[t]) (block indices relative to row/col kb + NB) -= L21 D L21^T, each as four
// chained v_mfma_f64_16x16x4_f64 (K = 16), accumulator initialised with the A block; the B operand is the staged L21
// scaled by D on the fly. The NT tiles' loads are issued together, so their L2 round trips overlap (the update is
// latency-bound at one workgroup per problem). to_cb: the tiles are the next block column (bc = 0), written to the
// block-column buffer (the next panel rows and diagonal block read them there) instead of back to A; upd = false:
// copied there without an update.
// Lane maps (gfx950, f64): A operand L[R0 + (lane&15)][k0 + (lane>>4)], B operand L[C0 + (lane&15)][k0 + (lane>>4)]
// D[k0 + (lane>>4)], C/D col = lane&15, row = (lane>>4) + 4 reg.
typedef double dbl4 __attribute__((ext_vector_type(4)));
template <int NT, bool to_cb>
__device__ __forceinline__ void ldlt_tiles16(gdouble* A, int N, int kb, const double* PL, const double* dkp, int m,
                                             double* CB, int cs, const int* br, const int* bc, bool upd, int lane) {
    const int col = lane & 15, rq = lane >> 4;
    dbl4 c[NT];
#pragma unroll
    for (int u = 0; u < NT; u++) {
        const int R0 = kb + NB + 16 * br[u], C0 = kb + NB + 16 * bc[u];
#pragma unroll
        for (int r = 0; r < 4; r++) c[u][r] = A[(size_t)(R0 + rq + 4 * r) * N + C0 + col];
    }
    if (upd) {
#pragma unroll
        for (int k0 = 0; k0 < NB; k0 += 4) {
            const int k = k0 + rq;
            const double dkk = dkp[k];
#pragma unroll
            for (int u = 0; u < NT; u++) {
                const double av = -PL[(size_t)k * m + 16 * br[u] + col];
                const double bv = PL[(size_t)k * m + 16 * bc[u] + col] * dkk;
                c[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c[u], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < NT; u++) {
        const int R0 = kb + NB + 16 * br[u], C0 = kb + NB + 16 * bc[u];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            if (to_cb) CB[(size_t)col * cs + 16 * br[u] + rq + 4 * r] = c[u][r];
            else A[(size_t)(R0 + rq + 4 * r) * N + C0 + col] = c[u][r];
        }
    }
}

// A wave's queue of non-zero tiles, flushed LDLT_BATCH at a time (wave-uniform: the tile ids and the tile mask are
// the same in every lane)
#ifndef MAM_LDLT_BATCH
#define MAM_LDLT_BATCH 4
#endif
constexpr int LDLT_BATCH = MAM_LDLT_BATCH;
template <bool to_cb>
struct TileQueue {
    int br[LDLT_BATCH], bc[LDLT_BATCH];
    int n = 0;
    __device__ __forceinline__ void push(gdouble* A, int N, int kb, const double* PL, const double* dkp, int m,
                                         double* CB, int cs, int r, int c, int lane) {
        br[n] = r;
        bc[n] = c;
        if (++n == LDLT_BATCH) {
            ldlt_tiles16<LDLT_BATCH, to_cb>(A, N, kb, PL, dkp, m, CB, cs, br, bc, true, lane);
            n = 0;
        }
    }
    __device__ __forceinline__ void flush(gdouble* A, int N, int kb, const double* PL, const double* dkp, int m,
                                          double* CB, int cs, int lane) {
        for (int u = 0; u < n; u++) ldlt_tiles16<1, to_cb>(A, N, kb, PL, dkp, m, CB, cs, br + u, bc + u, true, lane);
        n = 0;
    }
};


#ifdef MAM_LDLT_TRACE
// per-column timestamps of window 0 of the last k_ldlt_tiles launch (dataflow form): [kc][0..5] = after the critical
// flag wait, after the pulled updates, after the panel loads, after the pivot steps, after the flag set, backward
// step done
__device__ long long g_ltrace[40][8];
// (timestamps kept in LDS — sh.ltr — and copied out once at the end: a global store per point would put its own
// vmcnt wait into the next point's interval)
#define LTRACE(k, dep)                                                                          \
    do {                                                                                        \
        asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(dep) : "memory");                            \
        const long long tn_ = clock64();                                                        \
        if ((threadIdx.x & 63) == 0) sh.ltr[kc][k] = (int)tn_;                                  \
    } while (0)
#else
#define LTRACE(k, dep) \
    do {               \
    } while (0)
#endif

#ifdef MAM_LDLT_PROFILE
// cycles per phase summed over workgroups (thread 0 after each barrier): init, B, C1, C2, solve, diag (wave 0), -, WGs
__device__ unsigned long long g_lprof[8];
#define LPROF(k)                                                                     \
    do {                                                                             \
        if (t == 0) {                                                                \
            const long long tn = clock64();                                          \
            atomicAdd(&g_lprof[k], (unsigned long long)(tn - lp0));                  \
            lp0 = tn;                                                                \
        }                                                                            \
    } while (0)
#else
#define LPROF(k) \
    do {         \
    } while (0)
#endif

// grid (Q): with lookahead — after a panel's rows (B), the next block column is updated first (C1) into the
// block-column buffer CB (so the next diagonal block and panel rows read it from LDS, not back from A); then wave 0
// factors the next diagonal block while the other waves update the rest of the trailing matrix (C2). dk alternates
// between two slots: C2's trailing update reads the panel's D while wave 0 writes the next one.
#ifndef MAM_LDLT_C1_PF
#define MAM_LDLT_C1_PF 3
#endif
constexpr int C1_PF = MAM_LDLT_C1_PF;   // (C1) tiles per wave prefetched across (B)
constexpr int LDLT_TM_MAX = 40;         // the LDS path's tile-mask copy: nt <= 40 (npad <= 640)
// The factorization's static LDS, shared by both forms of k_ldlt (ldlt_global, ldlt_tiles)
struct LdltShared {
    // (the two forms' own fields share their LDS: a launch runs one form per problem. Every byte here is taken from
    // the tile pool's budget.)
    union {
        struct {
            double Ld[NB * NB];  // ldlt_global: L11 row-major
            double invdk[NB];
        };
        struct {
            // ldlt_tiles: per block column kc the rows r > kc of its non-zero tiles (ascending), per block row kc the
            // columns c < kc of its non-zero tiles — the panel / trailing / backward loops walk only those
            alignas(4) int8_t clist[40 * 40];
            alignas(4) int8_t rlist[40 * 40];
        };
    };
    double dk[2][NB];
    int fail;
    // ldlt_global<true>: the tile mask (uint8 [nt][nt]); ldlt_tiles: the tile slot map (int16 [nt][nt])
    int16_t map[LDLT_TM_MAX * LDLT_TM_MAX];
    uint8_t ccount[40];
    uint8_t rcount[40];
    // ldlt_tiles' dataflow form (a column's D: the diagonal of its factored diagonal tile): the columns' factored /
    // solved flags, the widest column's tile count
    int cflag[40];
    int bflag[40];
    int tcnt[40];                // dataflow tasks: the column's tile tasks done
    alignas(4) int8_t order[40]; // dataflow: the block columns in dependency-level order (k_struct_tiles)
#ifdef MAM_LDLT_TRACE
    int ltr[40][8];   // (low 32 bits of the cycle counter)
#endif
    int maxc;
};

// S factored in place in HBM with the panel / block-column workspace in LDS (use_lds) or in the problem's scratch: the
// form for problems whose non-zero tiles do not fit in LDS (dense covisibility, large windows)
template <bool use_lds>
__device__ __forceinline__ void ldlt_global(const Prob& d, double* lds_ws, LdltShared& sh) {
    LM& lm = *d.lm;
    const int n = 6 * d.Np, N = d.npad;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    gdouble* A = (gdouble*)d.S;   // global address space: its loads must not count in lgkmcnt (flat)
    double* ws = use_lds ? lds_ws : d.ws;
    const int cs = ldlt_cb_stride(N);
    double* PL = ws;
    double* CB = ws + (size_t)NB * (N - NB);
    double* Y = CB + (size_t)NB * cs;
    double* Ld = sh.Ld;
    double (*dk)[NB] = sh.dk;
    double* invdk = sh.invdk;
    int& fail = sh.fail;
    // the tile mask: the phases below test it before their loads, so its reads sit on their critical paths
    uint8_t* tm_lds = reinterpret_cast<uint8_t*>(sh.map);
    const uint8_t* tmask = use_lds ? tm_lds : d.tmask;
#ifdef MAM_LDLT_PROFILE
    long long lp0 = clock64();
#endif
    if (t == 0) fail = 0;
    if (use_lds)
        for (int q = t; q < d.nt * d.nt; q += LDLT_THREADS) tm_lds[q] = d.tmask[q];
    for (int i = t; i < N; i += LDLT_THREADS) {
        Y[i] = i < n ? d.bs[i] : 0.0;
        if (i >= n) A[(size_t)i * N + i] = 1.0;
    }
    __syncthreads();
    // block column 0 into CB (its non-zero tiles)
    for (int i = t; i < N; i += LDLT_THREADS) {
        if (!tmask[(size_t)(i / NB) * d.nt]) continue;
#pragma unroll
        for (int j = 0; j < NB; j++) CB[(size_t)j * cs + i] = A[(size_t)i * N + j];
    }
    __syncthreads();
    if (wid == 0) ldlt_diag(A, N, 0, CB, cs, Y, Ld, dk[0], invdk, &fail, lane);
    __syncthreads();
    LPROF(0);
    for (int kb = 0, p = 0; kb < N; kb += NB, p ^= 1) {
        // (B) panel rows: L21 = A21 L11^-T D^-1 (into A and, transposed, into PL), y2 -= L21 y1; A21 from CB
        const int m = N - kb - NB;
        const int kc = kb / NB;
        const uint8_t* tcol = tmask + kc;   // tcol[r * nt]: tile (r, kc) of L non-zero
        const uint8_t* ncol = tmask + kc + 1;   // tile (r, kc + 1) of L non-zero
        const double* dkp = dk[p];
        const int T16 = m / 16;
        const int i0 = kb + NB + t;
        const bool row0 = i0 < N && tcol[(size_t)(i0 / NB) * d.nt];
        // (C1)'s first tiles of this wave (br = wid + 8 u), loaded from A before (B): their L2 round trip overlaps it
        const int col16 = lane & 15, rq = lane >> 4;
        dbl4 pc[C1_PF];
#pragma unroll
        for (int u = 0; u < C1_PF; u++) {
            const int br = wid + (LDLT_THREADS / 64) * u;
            if (br < T16 && ncol[(size_t)(kc + 1 + br) * d.nt]) {
                const int R0 = kb + NB + 16 * br, C0 = kb + NB;
#pragma unroll
                for (int r = 0; r < 4; r++) pc[u][r] = A[(size_t)(R0 + rq + 4 * r) * N + C0 + col16];
            }
        }
        for (int i = i0; i < N; i += LDLT_THREADS) {
            // structurally zero row of L21: no update, no y change
            if (!(i == i0 ? row0 : tcol[(size_t)(i / NB) * d.nt] != 0)) continue;
            // keep the L11 factors in LDS (reading them per row): hoisting all 120 into registers spills
            asm volatile("" ::: "memory");
            double w[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) w[j] = CB[(size_t)j * cs + (i - kb)];
#pragma unroll
            for (int j = 1; j < NB; j++) {
#pragma unroll
                for (int k = 0; k < j; k++) w[j] = fma(-w[k], Ld[j * NB + k], w[j]);
            }
            double yi = Y[i];
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const double lij = w[j] * invdk[j];
                A[(size_t)i * N + kb + j] = lij;
                PL[(size_t)j * m + (i - kb - NB)] = lij;
                yi = fma(-lij, Y[kb + j], yi);
            }
            Y[i] = yi;
        }
        __syncthreads();
        LPROF(1);
        if (m == 0) break;
        // (C1) the next block column into CB: its non-zero tiles (br, 0), one wave each, updated where L(kc + 1 + br,
        // kc) and L(kc + 1, kc) are non-zero, copied otherwise
        {
            const bool c1nz = tcol[(size_t)(kc + 1) * d.nt] != 0;
#pragma unroll
            for (int u = 0; u < C1_PF; u++) {
                const int br = wid + (LDLT_THREADS / 64) * u;
                if (br >= T16 || !ncol[(size_t)(kc + 1 + br) * d.nt]) continue;
                if (c1nz && tcol[(size_t)(kc + 1 + br) * d.nt]) {
#pragma unroll
                    for (int k0 = 0; k0 < NB; k0 += 4) {
                        const int k = k0 + rq;
                        const double av = -PL[(size_t)k * m + 16 * br + col16];
                        const double bv = PL[(size_t)k * m + col16] * dkp[k];
                        pc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, pc[u], 0, 0, 0);
                    }
                }
#pragma unroll
                for (int r = 0; r < 4; r++) CB[(size_t)col16 * cs + 16 * br + rq + 4 * r] = pc[u][r];
            }
            TileQueue<true> tq;
            for (int br = wid + (LDLT_THREADS / 64) * C1_PF; br < T16; br += LDLT_THREADS / 64) {
                if (!ncol[(size_t)(kc + 1 + br) * d.nt]) continue;
                if (c1nz && tcol[(size_t)(kc + 1 + br) * d.nt]) {
                    tq.push(A, N, kb, PL, dkp, m, CB, cs, br, 0, lane);
                } else {
                    const int z = 0;
                    ldlt_tiles16<1, true>(A, N, kb, PL, dkp, m, CB, cs, &br, &z, false, lane);
                }
            }
            tq.flush(A, N, kb, PL, dkp, m, CB, cs, lane);
        }
        __syncthreads();
        LPROF(2);
        // (C2) wave 0 factors the next diagonal block; the other waves update the blocks with bc >= 1
        if (wid == 0) {
#ifdef MAM_LDLT_PROFILE
            const long long td = clock64();
#endif
            ldlt_diag(A, N, kb + NB, CB, cs, Y, Ld, dk[p ^ 1], invdk, &fail, lane);
#ifdef MAM_LDLT_PROFILE
            if (lane == 0) atomicAdd(&g_lprof[5], (unsigned long long)(clock64() - td));
#endif
        } else {
            const int T2 = T16 - 1;
            const int n2 = T2 * (T2 + 1) / 2;
            TileQueue<false> tq;
            for (int q = wid - 1; q < n2; q += LDLT_THREADS / 64 - 1) {
                int tr, tc;
                tri_index(q, &tr, &tc);
                if (tcol[(size_t)(kc + 2 + tr) * d.nt] && tcol[(size_t)(kc + 2 + tc) * d.nt])
                    tq.push(A, N, kb, PL, dkp, m, CB, cs, tr + 1, tc + 1, lane);
            }
            tq.flush(A, N, kb, PL, dkp, m, CB, cs, lane);
        }
        __syncthreads();
        LPROF(3);
    }
    if (t == 0) lm.fail = fail;
    if (fail) return;   // uniform (LDS flag after the last barrier)
    // y /= D
    for (int i = t; i < N; i += LDLT_THREADS) Y[i] /= A[(size_t)i * N + i];
    __syncthreads();
    // backward substitution L^T x = y: block solve by wave 0, then each thread i < kb updates its own y_i
    for (int kb = N - NB; kb >= 0; kb -= NB) {
        const bool pre = t < kb && tmask[(size_t)(kb / NB) * d.nt + t / NB];   // L(kb.., t) not structurally zero
        double a[NB];
        if (pre) {
#pragma unroll
            for (int j = 0; j < NB; j++) a[j] = A[(size_t)(kb + j) * N + t];
        }
        if (wid == 0) {
            double col[NB];   // lane c holds L(kb + j, kb + c) for j > c
#pragma unroll
            for (int j = 0; j < NB; j++) col[j] = lane < NB ? A[(size_t)(kb + j) * N + kb + lane] : 0.0;
            double v = lane < NB ? Y[kb + lane] : 0.0;
#pragma unroll
            for (int j = NB - 1; j >= 0; j--) {
                const double xj = bcast16_d(v, j);
                if (lane < j) v = fma(-col[j], xj, v);
            }
            if (lane < NB) Y[kb + lane] = v;
        }
        __syncthreads();
        // the first row's L column was loaded before the barrier, beside the block solve
        if (pre) {
            double sy = Y[t];
#pragma unroll
            for (int j = 0; j < NB; j++) sy = fma(-a[j], Y[kb + j], sy);
            Y[t] = sy;
        }
        for (int i = t + LDLT_THREADS; i < kb; i += LDLT_THREADS) {
            if (!tmask[(size_t)(kb / NB) * d.nt + i / NB]) continue;   // L(kb.., i) structurally zero
            double sy = Y[i];
#pragma unroll
            for (int j = 0; j < NB; j++) sy = fma(-A[(size_t)(kb + j) * N + i], Y[kb + j], sy);
            Y[i] = sy;
        }
        __syncthreads();
    }
    for (int i = t; i < n; i += LDLT_THREADS) d.x[6 * (size_t)d.iperm[i / 6] + i % 6] = Y[i];   // (pose order)
    LPROF(4);
#ifdef MAM_LDLT_PROFILE
    if (t == 0) atomicAdd(&g_lprof[7], 1ull);
#endif
}

// ---- the factorization with all of L in LDS (lm.tiles_lds: the structurally non-zero tiles + y fit the dynamic
// LDS). The tiles S holds (k_schur_blk: pose blocks, lower triangle) are loaded once into a pool of 16x16 tiles
// (k_struct_tiles' slots, tslot / tlist), factored there and never written back: only x leaves the workgroup. Blocked
// right-looking LDL^T with tile skipping: per block column k, tall panels (the diagonal tile and the column's
// non-zero tiles below it factored in one register pass, y's forward solve folded in), then the trailing tiles
// updated by f64 MFMA — column k + 1's first (what the next panel reads), the rest beside the next panel. No global
// memory round trip inside the panel loop.
// Tile layout: element (r, c) at c * 16 + (r ^ c) (column-major, rows XOR-swizzled by the column): the MFMA A / B
// operand reads (16 rows of one column per 16 lanes), the accumulator reads / writes (16 columns of one row) and the
// row-per-thread panel rows are all free of LDS bank conflicts within a 32-lane group.
// (tsw: see k_schur_blk)

// C(sc) -= L(sa) D L(sb)^T on tiles of the pool (one wave): four v_mfma_f64_16x16x4_f64, operands from LDS
__device__ __forceinline__ void tile_update(double* TL, int sc, int sa, int sb, const double* dkp, int lane) {
    const int col = lane & 15, rq = lane >> 4;
    double* C = TL + (size_t)sc * 256;
    const double* La = TL + (size_t)sa * 256;
    const double* Lb = TL + (size_t)sb * 256;
    dbl4 acc;
#pragma unroll
    for (int r = 0; r < 4; r++) acc[r] = C[tsw(rq + 4 * r, col)];
#pragma unroll
    for (int k0 = 0; k0 < NB; k0 += 4) {
        const int k = k0 + rq;
        const double av = -La[tsw(col, k)];
        const double bv = Lb[tsw(col, k)] * dkp[k];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) C[tsw(rq + 4 * r, col)] = acc[r];
}

// tile_update for N tiles that share the B operand L(sb) (the updates one column pulls from column j): every LDS load
// first, then the N MFMA chains interleaved, then the stores — one tile's latency instead of N in turn (the pointers
// may alias as far as the compiler knows, so separate tile_update calls run back to back). Per tile the same four
// MFMAs in the same order as tile_update.
// With yj: also y_kc -= L(kc, j) y_j for the lane's row il (L(kc, j) = L(sb)), the same sequential FMAs as the tall
// panel's panel-row forward update, its operands loaded with the tiles'.
template <int N>
__device__ __forceinline__ void tile_update_multi(double* TL, const int* sc, const int* sa, int sb, const double* dkp,
                                                  int lane, const double* yj = nullptr, double* yd = nullptr,
                                                  int dstride = 1) {
    const int col = lane & 15, rq = lane >> 4;
    const double* Lb = TL + (size_t)sb * 256;
    double bv[4], av[N][4], lv[NB], yv[NB];
    dbl4 acc[N];
    if (yj) {
#pragma unroll
        for (int k = 0; k < NB; k++) {
            lv[k] = Lb[tsw(col, k)];
            yv[k] = yj[k];
        }
    }
    // the negation on the shared B operand: (-a) b and a (-b) are the same product, bit for bit, and the A operands
    // load straight into registers (no per-tile wait for a negation); an absent tile (sa < 0, uniform) loads a valid
    // tile, so every load issues unconditionally and one wait covers them all
#pragma unroll
    for (int q = 0; q < 4; q++) bv[q] = -(Lb[tsw(col, 4 * q + rq)] * dkp[dstride * (4 * q + rq)]);
#pragma unroll
    for (int u = 0; u < N; u++) {
        const double* C = TL + (size_t)(sa[u] >= 0 ? sc[u] : sb) * 256;
        const double* La = TL + (size_t)(sa[u] >= 0 ? sa[u] : sb) * 256;
#pragma unroll
        for (int r = 0; r < 4; r++) acc[u][r] = C[tsw(rq + 4 * r, col)];
#pragma unroll
        for (int q = 0; q < 4; q++) av[u][q] = La[tsw(col, 4 * q + rq)];
    }
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
        for (int u = 0; u < N; u++)
            if (sa[u] >= 0) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u][q], bv[q], acc[u], 0, 0, 0);
    if (yj) {
        double v = *yd;
#pragma unroll
        for (int k = 0; k < NB; k++) v = fma(-lv[k], yv[k], v);
        *yd = v;
    }
#pragma unroll
    for (int u = 0; u < N; u++) {
        if (sa[u] < 0) continue;
        double* C = TL + (size_t)sc[u] * 256;
#pragma unroll
        for (int r = 0; r < 4; r++) C[tsw(rq + 4 * r, col)] = acc[u][r];
    }
}

// ---- tall panels: the panel tiles factored together with the diagonal tile, lane (g, i) = (lane >> 4, lane & 15)
// holding row i of the diagonal tile (the same row in all four 16-lane groups) and row i of panel tile g of the
// column. The right-looking steps that factor the diagonal tile then also produce the panel rows' L (l = A(p, J) / d_J,
// A(p, K) -= l A(K, J), A(K, J) broadcast from lane K of the lane's own group) and the forward solve of y for both, in
// one pass: no M = L11^-T D^-1, no MFMA panel product and no barrier between the diagonal and its panel. The diagonal
// rows and their y see exactly the arithmetic of diag16_factor + diag16_forward.
// acc -= (value of src in lane K of this lane's 16-lane row) * m, the negation as the DPP form's src1 modifier (no
// v_xor / v_mov pair for -m on the pivot chain). No hazard nop: in Tall16 every use's m waits on the pivot's
// reciprocal chain, which starts from a DPP read of the same src, so src's last VALU write is many instructions back.
template <int K>
__device__ __forceinline__ void fnmac_bcast16(double& acc, double src, double m) {
    asm("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(src), "v"(m), "n"(K));
}
template <int J, int K>
struct FnmacRow16 {
    __device__ __forceinline__ static void run(double* row, double a, double l) {
        fnmac_bcast16<K>(row[K], a, l);
        FnmacRow16<J, K + 1>::run(row, a, l);
    }
};
template <int J>
struct FnmacRow16<J, NB> {
    __device__ __forceinline__ static void run(double*, double, double) {}
};
template <int J>
struct FnmacRow16<J, NB + 1> {
    __device__ __forceinline__ static void run(double*, double, double) {}
};
// X = L11^-1 by columns in right-looking order (lane c: x[r] = X(r, c)): for J, x[R] -= L(R, J) x[J], R > J, with
// L(R, J) broadcast from lane R (row[J] there: loaded from LDS, no VALU write to wait on). Each x[R] sees the same
// updates in the same order as Inv16 (bit-identical), but consecutive DPP FMAs no longer share an accumulator.
template <int J, int R>
struct InvR16 {
    __device__ __forceinline__ static void run(double* x, const double* row) {
        fnmac_bcast16<R>(x[R], row[J], x[J]);
        InvR16<J, R + 1>::run(x, row);
    }
};
template <int J>
struct InvR16<J, NB> {
    __device__ __forceinline__ static void run(double* x, const double* row) { InvR16<J + 1, J + 2>::run(x, row); }
};
template <>
struct InvR16<NB - 1, NB> {
    __device__ __forceinline__ static void run(double*, const double*) {}
};
template <int J>
struct Tall16 {
    __device__ __forceinline__ static void run(double* dr, double* pr, double& yd, double& yp, double& dmine, int il) {
        const double a = dr[J];
        const double dj = bcast16_d(a, J);
        if (il == J) dmine = dj;
        // the pivot's reciprocal: v_rcp_f64 and one third-order correction inv0 (1 + e + e^2), e = 1 - dj inv0 (the
        // seed's error cubed: well under an ulp) — three dependent FMAs on the chain instead of four. A zero pivot
        // is not masked: it fails the factorization (sh.fail), whose L and y nothing reads.
        const double inv0 = __builtin_amdgcn_rcp(dj);
        const double e = fma(-dj, inv0, 1.0);
        const double inv = fma(inv0, fma(e, e, e), inv0);
        const double l = a * inv, lp = pr[J] * inv;
        const double yj = bcast16_d(yd, J);   // y_J final (steps 0 .. J - 1 applied)
        // the next pivot's column first, as a DPP move (independent of l: issued early) + a plain FMA: a dependent
        // v_fmac_f64_dpp takes ~40 cycles to its result on gfx950, the move + FMA pair ~16 (scripts/valu_probe.hip)
        if constexpr (J + 1 < NB) dr[J + 1] = fma(-l, bcast16_d(a, J + 1), dr[J + 1]);
        FnmacRow16<J, J + 2>::run(dr, a, l);
        FnmacRow16<J, J + 1>::run(pr, a, lp);
        if (il > J) {
            dr[J] = l;
            yd = fma(-l, yj, yd);
        }
        pr[J] = lp;
        yp = fma(-lp, yj, yp);
        Tall16<J + 1>::run(dr, pr, yd, yp, dmine, il);
    }
};
template <>
struct Tall16<NB> {
    __device__ __forceinline__ static void run(double*, double*, double&, double&, double&, int) {}
};
// Tall16 with two panel rows per lane (tiles g and g + 4 of a column with up to 8 panel tiles); the panel rows' y is
// not kept (the dataflow form's rows pull theirs)
template <int J>
struct Tall16x2 {
    __device__ __forceinline__ static void run(double* dr, double* pr, double* pq, double& yd, double& dmine, int il) {
        const double a = dr[J];
        const double dj = bcast16_d(a, J);
        if (il == J) dmine = dj;
        const double inv0 = __builtin_amdgcn_rcp(dj);
        const double e = fma(-dj, inv0, 1.0);
        const double inv = fma(inv0, fma(e, e, e), inv0);
        const double l = a * inv, lp = pr[J] * inv, lq = pq[J] * inv;
        const double yj = bcast16_d(yd, J);
        if constexpr (J + 1 < NB) dr[J + 1] = fma(-l, bcast16_d(a, J + 1), dr[J + 1]);
        FnmacRow16<J, J + 2>::run(dr, a, l);
        FnmacRow16<J, J + 1>::run(pr, a, lp);
        FnmacRow16<J, J + 1>::run(pq, a, lq);
        if (il > J) {
            dr[J] = l;
            yd = fma(-l, yj, yd);
        }
        pr[J] = lp;
        pq[J] = lq;
        Tall16x2<J + 1>::run(dr, pr, pq, yd, dmine, il);
    }
};
template <>
struct Tall16x2<NB> {
    __device__ __forceinline__ static void run(double*, double*, double*, double&, double&, int) {}
};

// One tall-panel item of block column kc: the diagonal tile + the column's non-zero tiles clist[kc][4 q + g] (g = 0..3)
// factored; the item-0 wave stores the diagonal tile (L below, D on it; the upper triangle is left to the inverse
// pass), dk and y_kc, every group its panel tile's L and y rows
__device__ __forceinline__ void tall_panel(double* TL, const int16_t* slot, int nt, int kc, int q, double* Y,
                                           LdltShared& sh, double* dkp, int lane) {
    const int g = lane >> 4, il = lane & 15, kb = NB * kc;
    const int ncl = sh.ccount[kc];
    const int ip = 4 * q + g;
    const int r = ip < ncl ? sh.clist[kc * 40 + ip] : -1;
    double* Td = TL + (size_t)slot[kc * nt + kc] * 256;
    double* Tp = TL + (size_t)slot[(r >= 0 ? r : kc) * nt + kc] * 256;
    double dr[NB], pr[NB];
#pragma unroll
    for (int c = 0; c < NB; c++) {
        dr[c] = Td[tsw(il, c)];
        pr[c] = r >= 0 ? Tp[tsw(il, c)] : 0.0;
    }
    double yd = Y[kb + il], yp = r >= 0 ? Y[NB * r + il] : 0.0;
    double dmine = 1.0;
    Tall16<0>::run(dr, pr, yd, yp, dmine, il);
    if (q == 0 && g == 0) {
#pragma unroll
        for (int c = 0; c < NB; c++)
            if (c <= il) Td[tsw(il, c)] = c < il ? dr[c] : dmine;
        dkp[il] = dmine;
        Y[kb + il] = yd;
        if (dmine == 0.0) sh.fail = 1;
    }
    if (r >= 0) {
#pragma unroll
        for (int c = 0; c < NB; c++) Tp[tsw(il, c)] = pr[c];
        Y[NB * r + il] = yp;
    }
}

// ---- dataflow form for banded tile patterns (every column has at most 4 non-zero tiles below its diagonal tile, so one
// tall-panel item per column): no workgroup barriers inside the factorization, the waves synchronise through LDS flags
// (the tasks: see flow_tile_task). The backward solve runs as one owner wave per column in reverse (column kc pulls
// L(r, kc)^T x_r from its rows r once their flags are set). Every tile and every y entry sees the same updates in the
// same order as in the right-looking schedule of ldlt_tiles (each update's inner sums split into two chains: the
// rounding differs from that schedule's in the last bits).
__device__ __forceinline__ int lds_flag_load(const int* f) {
    return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_flag_wait(const int* f) {
    while (!lds_flag_load(f)) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void lds_flag_set(int* f) {
    __hip_atomic_store(f, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The dataflow factorization as tasks: per block column kc, tile task t = 0 .. ncl pulls every update one tile of the
// column receives (t = 0 the diagonal tile, which also pulls y_kc; t = 1 + a the panel tile of row clist[kc][a]) — for
// each column j < kc with L(r, j) non-zero, in ascending j, T(r, kc) -= L(r, j) D_j L(kc, j)^T, waiting for column j's
// flag when it gets there — and counts itself done in tcnt[kc]; the panel task (t = FLOW_TPC - 1) waits for the count,
// factors the tall panel and sets the column's flag. Task (kc, t) runs on wave (FLOW_TPC kc + t) % NW: a column's
// tasks are on distinct waves, so once column kc - 1's flag is set the <= 5 tiles of column kc take their last update
// in parallel (4 f64 MFMAs each, 64 cycles apiece) instead of one wave's 16 in turn, and the next column's tile tasks
// are never on the wave factoring this column's panel. Every wave walks the columns in ascending order with at most
// one task per column (dependencies only on earlier columns, or on the same column's tile tasks: no wait cycle).
constexpr int FLOW_TPC = 10;   // up to 9 tile tasks + the panel task per column (columns of up to 8 panel tiles)

// C(sc) -= L(sa) D_j L(sb)^T for one tile (a tile task's pulled update), with WITH_Y also y_kc -= L(kc, j) y_j (lane
// il's row; L(kc, j) = L(sb)): every LDS operand loaded before any use (one wait instead of one per MFMA step), the four
// MFMAs as two independent chains of two summed at the end, the y dot product as two chains of eight
template <bool WITH_Y>
__device__ __forceinline__ void tile_update1(double* TL, int sc, int sa, int sb, const double* Dj, int lane,
                                             const double* yj, double& yd) {
    const int col = lane & 15, rq = lane >> 4;
    double* C = TL + (size_t)sc * 256;
    const double* La = TL + (size_t)sa * 256;
    const double* Lb = TL + (size_t)sb * 256;
    double a[4], b[4], dk[4], lv[NB], yv[NB];
    dbl4 acc, acc1;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        a[q] = La[tsw(col, 4 * q + rq)];
        b[q] = Lb[tsw(col, 4 * q + rq)];
        dk[q] = Dj[NB * (4 * q + rq)];   // D_j(k) = the diagonal of column j's factored diagonal tile, tsw(k, k)
    }
#pragma unroll
    for (int r = 0; r < 4; r++) acc[r] = C[tsw(rq + 4 * r, col)];
    if constexpr (WITH_Y) {
#pragma unroll
        for (int k = 0; k < NB; k++) {
            lv[k] = Lb[tsw(col, k)];
            yv[k] = yj[k];
        }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = 0; r < 4; r++) acc1[r] = 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], -(b[0] * dk[0]), acc, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[2], -(b[2] * dk[2]), acc1, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], -(b[1] * dk[1]), acc, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[3], -(b[3] * dk[3]), acc1, 0, 0, 0);
    if constexpr (WITH_Y) {
        double v0 = yd, v1 = 0.0;
#pragma unroll
        for (int k = 0; k < NB / 2; k++) v0 = fma(-lv[k], yv[k], v0);
#pragma unroll
        for (int k = NB / 2; k < NB; k++) v1 = fma(-lv[k], yv[k], v1);
        yd = v0 + v1;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) C[tsw(rq + 4 * r, col)] = acc[r] + acc1[r];
}

__device__ __forceinline__ void flow_tile_task(double* TL, const int16_t* slot, int nt, int kc, int t, double* Y,
                                               LdltShared& sh, int lane) {
    const int il = lane & 15, kb = NB * kc;
    const int nrl = __builtin_amdgcn_readfirstlane(sh.rcount[kc]);
    const int r = t == 0 ? kc : __builtin_amdgcn_readfirstlane(sh.clist[kc * 40 + t - 1]);
    const int sc = __builtin_amdgcn_readfirstlane(slot[r * nt + kc]);
    double yd = t == 0 ? Y[kb + il] : 0.0;
    for (int q = 0; q < nrl; q++) {
        const int j = __builtin_amdgcn_readfirstlane(sh.rlist[kc * 40 + q]);
        const int sb = __builtin_amdgcn_readfirstlane(slot[kc * nt + j]);
        const int sa = t == 0 ? sb : __builtin_amdgcn_readfirstlane(slot[r * nt + j]);
        if (sa < 0) continue;   // uniform: L(r, j) is zero
        lds_flag_wait(&sh.cflag[j]);
        if (t == 0) LTRACE(6, j);
        // y_kc -= L(kc, j) y_j rides on the diagonal tile's update
        const double* Dj = TL + (size_t)__builtin_amdgcn_readfirstlane(slot[j * nt + j]) * 256;
        if (t == 0)
            tile_update1<true>(TL, sc, sa, sb, Dj, lane, Y + NB * j, yd);
        else
            tile_update1<false>(TL, sc, sa, sb, Dj, lane, nullptr, yd);
    }
    if (t == 0) {
        if (lane < NB) Y[kb + lane] = yd;
        LTRACE(0, yd);
    }
    if (lane == 0) __hip_atomic_fetch_add(&sh.tcnt[kc], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void flow_panel_task(double* TL, const int16_t* slot, int nt, int kc, double* Y,
                                                LdltShared& sh, int lane) {
    const int g = lane >> 4, il = lane & 15, kb = NB * kc;
    const int ncl = __builtin_amdgcn_readfirstlane(sh.ccount[kc]);
    const int sd = __builtin_amdgcn_readfirstlane(slot[kc * nt + kc]);
    int rows[8], rsl[8];
#pragma unroll
    for (int a = 0; a < 8; a++) {
        rows[a] = a < ncl ? __builtin_amdgcn_readfirstlane(sh.clist[kc * 40 + a]) : -1;
        rsl[a] = a < ncl ? __builtin_amdgcn_readfirstlane(slot[rows[a] * nt + kc]) : -1;
    }
    while (__hip_atomic_load(&sh.tcnt[kc], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= ncl)
        __builtin_amdgcn_s_sleep(1);
#ifdef MAM_LDLT_PROFILE
    long long tp0 = clock64();
#endif
    LTRACE(1, kc);
    // the tall panel: the diagonal tile and the panel tiles, lane (g, il) with row il of tiles g (and g + 4)
    const int r = g == 0 ? rows[0] : g == 1 ? rows[1] : g == 2 ? rows[2] : rows[3];
    const int rs = g == 0 ? rsl[0] : g == 1 ? rsl[1] : g == 2 ? rsl[2] : rsl[3];
    double* Td = TL + (size_t)sd * 256;
    double* Tp = TL + (size_t)(r >= 0 ? rs : sd) * 256;
    double dr[NB], pr[NB];
    // (r is per 16-lane group: every lane loads — an absent panel tile reads the diagonal tile — and selects, no
    // exec-masked load per column)
#pragma unroll
    for (int c = 0; c < NB; c++) {
        dr[c] = Td[tsw(il, c)];
        pr[c] = Tp[tsw(il, c)];
    }
#pragma unroll
    for (int c = 0; c < NB; c++) pr[c] = r >= 0 ? pr[c] : 0.0;
    double yd = Y[kb + il], yp = 0.0, dmine = 1.0;
    const bool two = ncl > 4;   // uniform
    int r2 = -1;
    double* Tq = Td;
    double pq[NB];
    if (two) {
        r2 = g == 0 ? rows[4] : g == 1 ? rows[5] : g == 2 ? rows[6] : rows[7];
        const int rs2 = g == 0 ? rsl[4] : g == 1 ? rsl[5] : g == 2 ? rsl[6] : rsl[7];
        Tq = TL + (size_t)(r2 >= 0 ? rs2 : sd) * 256;
#pragma unroll
        for (int c = 0; c < NB; c++) pq[c] = Tq[tsw(il, c)];
#pragma unroll
        for (int c = 0; c < NB; c++) pq[c] = r2 >= 0 ? pq[c] : 0.0;
    }
    LTRACE(2, dr[15]);
#ifdef MAM_LDLT_PROFILE
    long long tp1 = clock64();
    if (lane == 0) atomicAdd(&g_lprof[6], (unsigned long long)(tp1 - tp0));   // the panel loads
#endif
    if (two)
        Tall16x2<0>::run(dr, pr, pq, yd, dmine, il);
    else
        Tall16<0>::run(dr, pr, yd, yp, dmine, il);
    LTRACE(3, dmine);
#ifdef MAM_LDLT_PROFILE
    long long tp2 = clock64();
    if (lane == 0) atomicAdd(&g_lprof[5], (unsigned long long)(tp2 - tp1));   // the tall panel's pivot steps
#endif
    // the whole row, unpredicated: c < il holds L, c == il the pivot (dr[il] is never updated at its own step), the
    // entries above the diagonal are overwritten by the L^-T pass below before anything reads them
    if (g == 0) {
#pragma unroll
        for (int c = 0; c < NB; c++) Td[tsw(il, c)] = dr[c];
        Y[kb + il] = yd;
        if (dmine == 0.0) sh.fail = 1;
    }
    if (r >= 0) {
#pragma unroll
        for (int c = 0; c < NB; c++) Tp[tsw(il, c)] = pr[c];
    }
    if (two && r2 >= 0) {
#pragma unroll
        for (int c = 0; c < NB; c++) Tq[tsw(il, c)] = pq[c];
    }
    lds_flag_set(&sh.cflag[kc]);
    LTRACE(4, kc);
#ifdef MAM_LDLT_PROFILE
    if (lane == 0) atomicAdd(&g_lprof[2], (unsigned long long)(clock64() - tp2));   // stores + flag
#endif
    // the diagonal tile's L^-T into its upper triangle (the backward solve's block), from the factored rows in registers
    // (lane R's dr[J] = L(R, J) for J < R): off the critical path, the next columns no longer read this tile's upper part
    if (g == 0) {
        double x[NB];
#pragma unroll
        for (int c = 0; c < NB; c++) x[c] = (c == il) ? 1.0 : 0.0;
        InvR16<0, 1>::run(x, dr);
#pragma unroll
        for (int c = 0; c < NB; c++)
            if (c > il) Td[tsw(il, c)] = x[c];
    }
}

// backward step of column kc (its owner wave): x_kc = L_kc^-T (y_kc / D_kc - sum_r L(r, kc)^T x_r), r over the column's
// non-zero tiles in descending order (the order the right-looking backward solve applied them in)
__device__ __forceinline__ void flow_back_column(const double* TL, const int16_t* slot, int nt, int kc, double* Y,
                                                 LdltShared& sh, int lane) {
    const int il = lane & 15, kb = NB * kc;
    const double* Td = TL + (size_t)slot[kc * nt + kc] * 256;
    double v = Y[kb + il] / Td[tsw(il, il)];
    for (int a = sh.ccount[kc] - 1; a >= 0; a--) {
        const int r = sh.clist[kc * 40 + a];
        lds_flag_wait(&sh.bflag[r]);
        const double* Tr = TL + (size_t)slot[r * nt + kc] * 256;
        const double* xr = Y + NB * r;
        double sy1 = 0.0;
#pragma unroll
        for (int j = 0; j < NB / 2; j++) v = fma(xr[j], -Tr[tsw(j, il)], v);   // y_i -= L(r + j, i) x_j: two partial
#pragma unroll                                                                  // chains of 8 (j < 8, j >= 8)
        for (int j = NB / 2; j < NB; j++) sy1 = fma(xr[j], -Tr[tsw(j, il)], sy1);
        v += sy1;
    }
    // x_b = L11^-T y_b from the upper triangle the factor step wrote; y_j from lane j of the lane's own 16-lane row
    // (every row holds the block's y) by DPP
    double w = v, w1 = 0.0;
#pragma unroll
    for (int j = 1; j < NB / 2; j++) {
        const double f = fma(Td[tsw(il, j)], bcast16_d(v, j), w);
        w = j > il ? f : w;
    }
#pragma unroll
    for (int j = NB / 2; j < NB; j++) {
        const double f = fma(Td[tsw(il, j)], bcast16_d(v, j), w1);
        w1 = j > il ? f : w1;
    }
    w += w1;
    if (lane < NB) Y[kb + lane] = w;
    lds_flag_set(&sh.bflag[kc]);
    LTRACE(5, w);
}

__device__ __forceinline__ void ldlt_tiles(const Prob& d, double* lds, LdltShared& sh, const LMHead& hd) {
    LM& lm = *d.lm;
    const int n = 6 * d.Np, N = d.npad, nt = d.nt, T = hd.ntiles;
    const int t = threadIdx.x, lane = t & 63, wid = __builtin_amdgcn_readfirstlane(t >> 6);   // uniform: scalar task branches
    constexpr int NW = LDLT_THREADS / 64;
#ifdef MAM_LDLT_PROFILE
    long long lp0 = clock64();
#endif
    double* TL = lds;                           // [T][256]
    double* Y = lds + (size_t)T * 256;          // [N]
    int16_t* slot = sh.map;                     // [nt][nt]
    // the prologue's global reads — the slot map, the column / row lists and counts k_struct_tiles made, y, and the
    // tile pool k_schur_blk wrote in slot order and LDS layout (padding identity included) — all issued before the
    // first LDS store, as global (not flat) loads: one memory round trip instead of one per small copy loop
    {
        typedef __attribute__((address_space(1))) const int16_t gi16;
        typedef __attribute__((address_space(1))) const uint32_t gu32;
        typedef __attribute__((address_space(1))) const uint8_t gu8;
        typedef __attribute__((address_space(1))) const double gd;
        constexpr int SPT = (LDLT_TM_MAX * LDLT_TM_MAX + LDLT_THREADS - 1) / LDLT_THREADS;
        constexpr int LPT = (LDLT_TM_MAX * 40 / 4 + LDLT_THREADS - 1) / LDLT_THREADS;
        constexpr int YPT = (LDLT_TM_MAX * NB + LDLT_THREADS - 1) / LDLT_THREADS;
        const int nn = nt * nt, nw = nt * 10;
        int16_t sv[SPT];
        uint32_t cw[LPT], rw[LPT];
        uint8_t cv = 0;
        double yv[YPT];
        // the pool: LDS-DMA (global_load_lds, 16 bytes per lane: one wave instruction fills 1 KB of the contiguous
        // image, no VGPRs), 1-KB chunks dealt to the waves
        {
            typedef __attribute__((address_space(1))) void gvoid;
            typedef __attribute__((address_space(3))) void lvoid;
            for (int c = wid; c < 2 * T; c += NW)
                __builtin_amdgcn_global_load_lds((gvoid*)(d.pool + (size_t)c * 128 + 2 * lane), (lvoid*)(TL + (size_t)c * 128),
                                                 16, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < SPT; u++) sv[u] = t + u * LDLT_THREADS < nn ? ((gi16*)d.tslot)[t + u * LDLT_THREADS] : 0;
#pragma unroll
        for (int u = 0; u < LPT; u++) {
            const int q = t + u * LDLT_THREADS;
            cw[u] = q < nw ? ((gu32*)d.clist_g)[q] : 0u;
            rw[u] = q < nw ? ((gu32*)d.rlist_g)[q] : 0u;
        }
        if (t < 2 * nt) cv = ((gu8*)d.ccnt_g)[t];
        const int8_t ov = t < nt ? ((__attribute__((address_space(1))) const int8_t*)d.order_g)[t] : 0;
#pragma unroll
        for (int u = 0; u < YPT; u++) {
            const int i = t + u * LDLT_THREADS;
            yv[u] = i < n ? ((gd*)d.bs)[i] : 0.0;
        }
        if (t == 0) {
            sh.fail = 0;
            sh.maxc = hd.maxc;
        }
#pragma unroll
        for (int u = 0; u < SPT; u++)
            if (t + u * LDLT_THREADS < nn) slot[t + u * LDLT_THREADS] = sv[u];
#pragma unroll
        for (int u = 0; u < LPT; u++) {
            const int q = t + u * LDLT_THREADS;
            if (q < nw) {
                reinterpret_cast<uint32_t*>(sh.clist)[q] = cw[u];
                reinterpret_cast<uint32_t*>(sh.rlist)[q] = rw[u];
            }
        }
        if (t < nt) {
            sh.ccount[t] = cv;
            sh.order[t] = ov;
            sh.cflag[t] = 0;
            sh.bflag[t] = 0;
            sh.tcnt[t] = 0;
        } else if (t < 2 * nt) {
            sh.rcount[t - nt] = cv;
        }
#pragma unroll
        for (int u = 0; u < YPT; u++)
            if (t + u * LDLT_THREADS < N) Y[t + u * LDLT_THREADS] = yv[u];
    }
    __syncthreads();
    LPROF(0);
#ifndef MAM_LDLT_FLOW
#define MAM_LDLT_FLOW 1
#endif
    if (MAM_LDLT_FLOW && sh.maxc <= 8 && nt <= 40) {   // uniform: every column one tall-panel item
        // the columns in dependency-level order (k_struct_tiles: a topological order, so every wave walking it
        // in turn waits only on tasks earlier in it), position sp's tasks on waves FLOW_TPC sp + t
        for (int sp = 0; sp < nt; sp++) {
            const int kc = __builtin_amdgcn_readfirstlane(sh.order[sp]);
            const int ncl = __builtin_amdgcn_readfirstlane(sh.ccount[kc]);
            // this wave's tasks of column kc in task order (tile tasks before the panel task: a wave holding both
            // finishes its tile task first)
            for (int tk = (wid - FLOW_TPC * sp % NW + NW) % NW; tk < FLOW_TPC; tk += NW) {
                if (tk == FLOW_TPC - 1)
                    flow_panel_task(TL, slot, nt, kc, Y, sh, lane);
                else if (tk <= ncl)
                    flow_tile_task(TL, slot, nt, kc, tk, Y, sh, lane);
            }
        }
        __syncthreads();
        LPROF(1);
        const int fl = sh.fail;
        if (t == 0) lm.fail = fl;
        if (fl) return;   // uniform
        // the backward steps in the reverse order (column kc waits for the rows below it: later in the order)
        for (int sp = nt - 1; sp >= 0; sp--)
            if (sp % NW == wid) flow_back_column(TL, slot, nt, __builtin_amdgcn_readfirstlane(sh.order[sp]), Y, sh, lane);
        __syncthreads();
        for (int i = t; i < n; i += LDLT_THREADS) d.x[6 * (size_t)d.iperm[i / 6] + i % 6] = Y[i];   // (pose order)
#ifdef MAM_LDLT_TRACE
        if (blockIdx.x == 0)
            for (int i = t; i < nt * 8; i += LDLT_THREADS) g_ltrace[i / 8][i % 8] = sh.ltr[i / 8][i % 8];
#endif
        LPROF(4);
#ifdef MAM_LDLT_PROFILE
        if (t == 0) atomicAdd(&g_lprof[7], 1ull);
#endif
        return;
    }
    // per block column kc, phase A: the tall-panel items of column kc (waves 0 ..) beside the rest of column kc - 1's
    // trailing update (the tiles (r, c), c >= kc + 1, by the other waves first); barrier; phase B (when L(kc + 1, kc) is
    // non-zero): column kc + 1's tiles updated by L(., kc) — what the next panel reads; barrier. Every tile still sees
    // its panels' updates in panel order.
    for (int kc = 0; kc < nt; kc++) {
        const int ncl = sh.ccount[kc];
        const int np = (ncl + 3) / 4 > 0 ? (ncl + 3) / 4 : 1;
#ifdef MAM_LDLT_PROFILE
        const long long td = clock64();
#endif
        for (int q = wid; q < np; q += NW) tall_panel(TL, slot, nt, kc, q, Y, sh, sh.dk[kc & 1], lane);
#ifdef MAM_LDLT_PROFILE
        if (t == 0) atomicAdd(&g_lprof[5], (unsigned long long)(clock64() - td));
#endif
        if (kc > 0) {   // column kc - 1's pairs (a >= b) whose column c = clist[b] >= kc + 1
            const int kp = kc - 1, nclp = sh.ccount[kp];
            const int b0 = (nclp > 0 && sh.clist[kp * 40] == kc) ? 1 : 0;
            const int m = nclp - b0, n2 = m * (m + 1) / 2;
            for (int i = (wid - np % NW + NW) % NW; i < n2; i += NW) {
                int a, b;
                tri_index(i, &a, &b);
                const int r = sh.clist[kp * 40 + a + b0], c = sh.clist[kp * 40 + b + b0];
                tile_update(TL, slot[r * nt + c], slot[r * nt + kp], slot[c * nt + kp], sh.dk[kp & 1], lane);
            }
        }
        __syncthreads();
        LPROF(1);
        if (kc + 1 == nt) break;
        if (ncl > 0 && sh.clist[kc * 40] == kc + 1) {   // uniform
            const int sb = slot[(kc + 1) * nt + kc];
            for (int a = wid; a < ncl; a += NW) {
                const int r = sh.clist[kc * 40 + a];
                tile_update(TL, slot[r * nt + kc + 1], slot[r * nt + kc], sb, sh.dk[kc & 1], lane);
            }
            __syncthreads();
        }
        LPROF(3);
    }
    const int fl = sh.fail;
    if (t == 0) lm.fail = fl;
    if (fl) return;   // uniform (LDS flag after the last barrier)
    // the diagonal tiles' L^-T into their upper triangles (the backward solve's blocks): one tile per 16-lane group
    {
        const int g = lane >> 4, il = lane & 15;
        for (int k0 = 4 * wid; k0 < nt; k0 += 4 * NW) {
            const int kc = k0 + g;
            if (kc >= nt) continue;   // uniform per 16-lane group (the DPP rows)
            double* Td = TL + (size_t)slot[kc * nt + kc] * 256;
            double row[NB], x[NB];
#pragma unroll
            for (int c = 0; c < NB; c++) {
                row[c] = Td[tsw(il, c)];
                x[c] = (c == il) ? 1.0 : 0.0;
            }
            InvR16<0, 1>::run(x, row);
#pragma unroll
            for (int c = 0; c < NB; c++)
                if (c > il) Td[tsw(il, c)] = x[c];
        }
    }
    __syncthreads();
    // y /= D and the backward substitution L^T x = y by wave 0 alone (a wave's LDS accesses complete in order, so no
    // barrier): per block x_b = L11^-T y_b from the diagonal tile's upper triangle (written by the inverse pass), then
    // y_i -= L(kb.., i)^T x_b for the rows i of the block row's non-zero tiles, four tiles per pass
    if (wid != 0) return;
    for (int i = lane; i < N; i += 64) {
        const int ii = i / NB;
        Y[i] /= TL[(size_t)slot[ii * nt + ii] * 256 + tsw(i & 15, i & 15)];
    }
    const int g = lane >> 4, il = lane & 15;
    for (int kc = nt - 1; kc >= 0; kc--) {
        const int kb = NB * kc;
        // x_b in every 16-lane row (the same arithmetic in each), so the update below takes x_j from lane j of its own
        // row by DPP instead of an LDS round trip
        const double* Td = TL + (size_t)slot[kc * nt + kc] * 256;
        double v = Y[kb + il];
        // predicated, not branched: every lane's loads issue together (a branch per j was one LDS round trip each);
        // two independent partial sums (j < 8, j >= 8) halve the dependent FMA chain (~10 cycles a link)
        double v1 = 0.0;
#pragma unroll
        for (int j = 1; j < NB / 2; j++) {
            const double f = fma(Td[tsw(il, j)], Y[kb + j], v);
            v = j > il ? f : v;
        }
#pragma unroll
        for (int j = NB / 2; j < NB; j++) {
            const double f = fma(Td[tsw(il, j)], Y[kb + j], v1);
            v1 = j > il ? f : v1;
        }
        v += v1;
        if (lane < NB) Y[kb + lane] = v;
        const int nrl = sh.rcount[kc];
        // x_j in every lane of the row by DPP moves once per block, then plain FMAs
        double xb[NB];
#pragma unroll
        for (int j = 0; j < NB; j++) xb[j] = bcast16_d(v, j);
        for (int i0 = 0; i0 < nrl; i0 += 4) {
            const int i = i0 + g;
            const int c = i < nrl ? sh.rlist[kc * 40 + i] : -1;   // L(kb.., 16 c..) not structurally zero
            const int s = c >= 0 ? slot[kc * nt + c] : slot[kc * nt + kc];   // (a valid tile; result unused)
            const double* Tr = TL + (size_t)s * 256;
            const int yi = NB * (c >= 0 ? c : kc) + il;
            double mt[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) mt[j] = -Tr[tsw(j, il)];
            double sy = Y[yi];
#pragma unroll
            for (int j = 0; j < NB / 2; j++) sy = fma(xb[j], mt[j], sy);   // sy -= L(kb + j, yi) x_j: two partial
            double sy1 = 0.0;                                               // chains of 8 (j < 8, j >= 8)
#pragma unroll
            for (int j = NB / 2; j < NB; j++) sy1 = fma(xb[j], mt[j], sy1);
            sy += sy1;
            if (c >= 0) Y[yi] = sy;
        }
    }
    for (int i = lane; i < n; i += 64) d.x[6 * (size_t)d.iperm[i / 6] + i % 6] = Y[i];   // (pose order)
    LPROF(4);
#ifdef MAM_LDLT_PROFILE
    if (t == 0) atomicAdd(&g_lprof[7], 1ull);
#endif
}

// Eigen Quaterniond(Matrix3d)
__device__ __forceinline__ void rot_to_quat(const double m[9], double q[4]) {
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
        if (m[8] > (i == 1 ? m[4] : m[0])) i = 2;
        // the three cases with constant indices (no dynamically indexed arrays: they would live in scratch)
        auto one = [&](auto I) {
            constexpr int ii = decltype(I)::value, jj = (ii + 1) % 3, kk = (jj + 1) % 3;
            double s = sqrt(m[3 * ii + ii] - m[3 * jj + jj] - m[3 * kk + kk] + 1.0);
            q[ii] = 0.5 * s;
            s = 0.5 / s;
            q[3] = (m[3 * kk + jj] - m[3 * jj + kk]) * s;
            q[jj] = (m[3 * jj + ii] + m[3 * ii + jj]) * s;
            q[kk] = (m[3 * kk + ii] + m[3 * ii + kk]) * s;
        };
        if (i == 0) one(std::integral_constant<int, 0>{});
        else if (i == 1) one(std::integral_constant<int, 1>{});
        else one(std::integral_constant<int, 2>{});
    }
}

__device__ __forceinline__ void normalize_q(double q[4]) {
    if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}

// O = exp(u) * T (VertexSE3Expmap::oplusImpl: SE3Quat::exp of the 6-vector, se3quat.h, then the product)
__device__ __forceinline__ void se3_exp_mul(const double u[6], const double* T, double* O) {
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double Om[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double Om2[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++)
            Om2[3 * r + c] = Om[3 * r] * Om[c] + Om[3 * r + 1] * Om[3 + c] + Om[3 * r + 2] * Om[6 + c];
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

// ================================================================================== fused per-trial point kernels
// A trial is k_point_sys -> k_schur_blk -> the factorization (+ its pose epilogue) -> k_point_trial -> k_ctl_end. The
// point kernels give one wave PW consecutive points and the slots of their edges (pe_idx, edge order within a point):
// lanes take slots for the per-edge work and lanes < PW take points for the per-point sums, handing over through LDS
// inside the wave, where the separate kernels of before (linearize, sys, schur_prep / backsub_update, trial
// linearize) each paid a launch and its dependent global round trips.
#ifndef MAM_PW
#define MAM_PW 8
#endif
constexpr int PW = MAM_PW;   // points per wave (a window's points have <= 8 observations: one 64-slot chunk)
#ifndef MAM_PW_SMALL
#define MAM_PW_SMALL 2
#endif
// lone windows of many observations per point: 2 points per wave (4x the point workgroups of its few trial kernels,
// each with a quarter of the dependent work; run_batch's choice)
constexpr int PW_SMALL = MAM_PW_SMALL;
static_assert((PW == 2 || PW == 4 || PW == 8) && (PW_SMALL == 2 || PW_SMALL == 4 || PW_SMALL == 8),
              "the point kernels are instantiated for 2, 4 and 8 points per workgroup");

// S's pose part at an iteration start: H_pp, b_p of Hessian pose block h — k_sys's sums (lanes strided over the pose's
// edge list in edge order, the same products, the same fixed-order wave reduction) on Jacobian terms recomputed from
// the state by the same linearisation (bit-identical to the records the point waves of the same launch write)
__device__ __forceinline__ void pose_sys_wave(const Prob& d, int h, int part, const double* pose, const double* pts) {
    const int lane = threadIdx.x;
    double acc[27];
#pragma unroll
    for (int k = 0; k < 27; k++) acc[k] = 0.0;
    // this partial's slots: chunks part, part + POSE_SPLIT, ... of 64 of the pose's edge list
    const int qs0 = d.qe_off[h], qs1 = d.qe_off[h + 1];
    for (int base = qs0 + 64 * part + lane; base < qs1; base += 64 * POSE_SPLIT * SYS_PF) {
        int qi[SYS_PF];
#pragma unroll
        for (int u = 0; u < SYS_PF; u++)
            qi[u] = base + 64 * POSE_SPLIT * u < qs1 ? d.qe_idx[base + 64 * POSE_SPLIT * u] : -1;
#pragma unroll
        for (int u = 0; u < SYS_PF; u++) {
            if (qi[u] < 0) break;
            const int e = qi[u], ipose = d.edge_pose[e];
            double j[21], hr[18];
            linearize_edge_at(d, pose + 7 * (size_t)ipose, pts + 3 * (size_t)d.edge_point[e], ipose, e, true, false, j,
                              hr);
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
    }
    double tot[7];
    {
        double v28[28];
#pragma unroll
        for (int k = 0; k < 27; k++) v28[k] = acc[k];
        v28[27] = 0.0;
        wave_sum_scatter4<7>(v28, tot);
    }
    const int g = lane >> 4, il = lane & 15;
    double val = 0.0;
#pragma unroll
    for (int i = 0; i < 7; i++) val = (il == i) ? tot[i] : val;
    const int q = 7 * g + il;
    if (il < 7 && q < 27) {
        if (q < 21) {
            int a = 0, r = q;
            while (r >= 6 - a) { r -= 6 - a; a++; }
            const int c = a + r;
            double* H = d.Hpp + 36 * ((size_t)part * d.Np + h);
            H[6 * a + c] = val;
            H[6 * c + a] = val;
        } else {
            d.bp[6 * ((size_t)part * d.Np + h) + (q - 21)] = val;
        }
    }
}

// D = H_ll + lambda I and its inverse as point_dinv computes it, from H in registers
__device__ __forceinline__ void dinv_of(const double H[9], double lambda, double o[9]) {
    double m[9];
#pragma unroll
    for (int k = 0; k < 9; k++) m[k] = H[k] + ((k % 4 == 0) ? lambda : 0.0);
    const double c00 = m[4] * m[8] - m[5] * m[7], c10 = m[7] * m[2] - m[8] * m[1], c20 = m[1] * m[5] - m[2] * m[4];
    const double det = c00 * m[0] + (c10 * m[3] + c20 * m[6]);
    const double inv = 1.0 / det;
    o[0] = c00 * inv; o[1] = c10 * inv; o[2] = c20 * inv;
    o[3] = (m[5] * m[6] - m[3] * m[8]) * inv; o[4] = (m[8] * m[0] - m[6] * m[2]) * inv;
    o[5] = (m[2] * m[3] - m[0] * m[5]) * inv;
    o[6] = (m[3] * m[7] - m[4] * m[6]) * inv; o[7] = (m[6] * m[1] - m[7] * m[0]) * inv;
    o[8] = (m[0] * m[4] - m[1] * m[3]) * inv;
}

// grid (ceil(L / PW) + Np POSE_SPLIT, Q) x 64, the start of every trial:
//  point waves — at an iteration start (need_lin, unless the setup pass already built iteration 0's system) the slots'
//    edges linearised (H_pl records, errors) and the points' H_ll, b_l summed in edge order from the slots' terms
//    (k_sys's sums); every trial D^-1 = (H_ll + lambda I)^-1 per point and, per slot, W = H_pl D^-1 and the
//    coefficients H_pl D^-1 b_l (k_schur_prep's products);
//  pose waves — at an iteration start H_pp, b_p in POSE_SPLIT partial sums per pose (pose_sys_wave).
template <int PWT>
__device__ __forceinline__ void point_sys_body(const Prob& d, const LMHead& hd) {
    if (hd.status || hd.done) return;
    const bool lin = hd.need_lin && !hd.sys_ready;
    const int nbp = (d.L + PWT - 1) / PWT;
    const double* pose = d.pose[hd.cur];
    const double* pts = d.pt[hd.cur];
    if ((int)blockIdx.x >= nbp) {
        const int h = (blockIdx.x - nbp) / POSE_SPLIT, part = (blockIdx.x - nbp) % POSE_SPLIT;
        if (lin && h < d.Np) pose_sys_wave(d, h, part, pose, pts);
        return;
    }
    const int lane = threadIdx.x;
    const double lambda = trial_lambda(hd);
    const int h0 = blockIdx.x * PWT, h1 = min(d.L, h0 + PWT);
    const int s0 = d.pe_off[h0], s1 = d.pe_off[h1];
    const bool one = s1 - s0 <= 64;   // one slot chunk: the slots' H_pl stay in registers for the W products
    __shared__ double cs[64 * 12];    // per slot: its H_ll (9) and b_l (3) terms
    __shared__ double pdv[PWT * 12];   // per point: D^-1 (9), D^-1 b_l (3)
    const int hl = h0 + lane;
    const bool plane = lane < PWT && hl < h1;
    const int ps0 = plane ? d.pe_off[hl] : 0, ps1 = plane ? d.pe_off[hl + 1] : 0;
    double H[9], bl[3], hr[18];
#pragma unroll
    for (int k = 0; k < 9; k++) H[k] = 0.0;
#pragma unroll
    for (int k = 0; k < 3; k++) bl[k] = 0.0;
#pragma unroll
    for (int k = 0; k < 18; k++) hr[k] = 0.0;
    // one chunk: the lane's slot edge loaded once, up front
    const int e1 = (one && s0 + lane < s1) ? d.pe_idx[s0 + lane] : 0;

    if (lin) {
        for (int c0 = s0; c0 < s1; c0 += 64) {
            const int s = c0 + lane;
            if (s < s1) {
                const int e = one ? e1 : d.pe_idx[s];
                double jr[21];
                linearize_edge(d, pose, pts, e, true, jr, hr);
                double* HP = d.hpl + 18 * (size_t)e;
#pragma unroll
                for (int k = 0; k < 18; k++) HP[k] = hr[k];
                const double wo = jr[20];
                double* c = cs + 12 * lane;
#pragma unroll
                for (int a = 0; a < 3; a++) {
                    c[9 + a] = jr[a] * jr[18] + jr[3 + a] * jr[19];
#pragma unroll
                    for (int cc = 0; cc < 3; cc++) c[3 * a + cc] = jr[a] * wo * jr[cc] + jr[3 + a] * wo * jr[3 + cc];
                }
            }
            __syncthreads();
            if (plane) {
                const int a0 = max(ps0, c0), a1 = min(ps1, c0 + 64);
                for (int q = a0; q < a1; q++) {
                    const double* c = cs + 12 * (q - c0);
#pragma unroll
                    for (int k = 0; k < 9; k++) H[k] += c[k];
#pragma unroll
                    for (int a = 0; a < 3; a++) bl[a] += c[9 + a];
                }
            }
            __syncthreads();
        }
    }
    if (plane) {
        double* Hg = d.Hll + 9 * (size_t)hl;
        double* bg = d.b + 6 * (size_t)d.Np + 3 * (size_t)hl;
        if (lin) {
#pragma unroll
            for (int k = 0; k < 9; k++) Hg[k] = H[k];
#pragma unroll
            for (int k = 0; k < 3; k++) bg[k] = bl[k];
        } else {
#pragma unroll
            for (int k = 0; k < 9; k++) H[k] = Hg[k];
#pragma unroll
            for (int k = 0; k < 3; k++) bl[k] = bg[k];
        }
        double Di[9];
        dinv_of(H, lambda, Di);
        double* Dg = d.Dinv + 9 * (size_t)hl;
        double* pv = pdv + 12 * lane;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            Dg[k] = Di[k];
            pv[k] = Di[k];
        }
#pragma unroll
        for (int i = 0; i < 3; i++) pv[9 + i] = Di[3 * i] * bl[0] + Di[3 * i + 1] * bl[1] + Di[3 * i + 2] * bl[2];
    }
    __syncthreads();
    for (int c0 = s0; c0 < s1; c0 += 64) {
        const int s = c0 + lane;
        if (s >= s1) continue;
        const int e = one ? e1 : d.pe_idx[s];
        const int4 em = d.emeta[e];
        double o[18], cf[6];
#pragma unroll
        for (int k = 0; k < 18; k++) o[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 6; k++) cf[k] = 0.0;
        if (em.y >= 0) {
            double B[18];
            if (lin && one) {
#pragma unroll
                for (int k = 0; k < 18; k++) B[k] = hr[k];
            } else if (lin) {   // several chunks: the H_pl record again by the same linearisation (not a reload of a
                double jr[21];  // line another wave of this launch may have cached before it was written)
                linearize_edge_at(d, pose + 7 * (size_t)d.edge_pose[e], pts + 3 * (size_t)em.x, d.edge_pose[e], e, true,
                                  false, jr, B);
            } else {
                const double* HP = d.hpl + 18 * (size_t)e;
#pragma unroll
                for (int k = 0; k < 18; k++) B[k] = HP[k];
            }
            const double* Di = pdv + 12 * (em.x - h0);
            const double* db = Di + 9;
#pragma unroll
            for (int i = 0; i < 6; i++) {
#pragma unroll
                for (int j = 0; j < 3; j++)
                    o[3 * i + j] = B[3 * i] * Di[j] + B[3 * i + 1] * Di[3 + j] + B[3 * i + 2] * Di[6 + j];
                cf[i] = B[3 * i] * db[0] + B[3 * i + 1] * db[1] + B[3 * i + 2] * db[2];
            }
        }
        double* W = d.bdinv + 18 * (size_t)e;
        double* C = d.coef + 6 * (size_t)e;
#pragma unroll
        for (int k = 0; k < 18; k++) W[k] = o[k];
#pragma unroll
        for (int k = 0; k < 6; k++) C[k] = cf[k];
    }
}

// the trial's chi2 and computeScale (levenberg.cpp:187-194: sum_j x_j (lambda x_j + b_j) over the full x) from
// k_point_trial's per-wave partials (fixed order: strided over RED virtual threads, then a tree; the same bits for any
// T) and the factorization epilogue's pose part
template <int T>
__device__ void trial_sums(const Prob& d, double* s, double* tempChi, double* scale0) {
    const int nbp = (d.L + d.pw - 1) / d.pw;   // k_point_trial's workgroups (d.pw points each)
    double acc[RED / T], acs[RED / T];
#pragma unroll
    for (int v = 0; v < RED / T; v++) {
        acc[v] = 0.0;
        acs[v] = 0.0;
        for (int j = threadIdx.x + T * v; j < nbp; j += RED) {
            acc[v] += d.part[j];
            acs[v] += d.part_s[j];
        }
    }
    *tempChi = block_sum<T>(acc, s);
    *scale0 = block_sum<T>(acs, s) + d.lm->scale_p;
}

// The end of a trial (thread 0): levenberg.cpp:108-158 (rho, accept / reject, lambda), then the iteration-end tests of
// levenberg.cpp:159-168 and sparse_optimizer.cpp:381-409, on the state lm (hd: its head as the trial left it)
__device__ void ctl_step(LM& lm, const LMHead& hd, double tempChi, double scale0) {
    const bool begin = hd.need_lin != 0;
    const double lambda = trial_lambda(hd);
    if (begin) {
        if (hd.its == 0) {
            lm.currentChi = lm.initialChi;
            lm.ni = 2.0;
            lm.nBad = 0;
        } else {
            lm.currentChi = lm.acceptedChi;
        }
        lm.iniChi = lm.currentChi;
        lm.qmax = 0;
        lm.need_lin = 0;
    }
    if (hd.fail) tempChi = DBL_MAX;
    double rho = lm.currentChi - tempChi;
    const double scale = scale0 + 1e-3;
    rho /= scale;
    if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow((2 * rho - 1), 3);
        alpha = fmin(alpha, 2. / 3.);
        const double scaleFactor = fmax(1. / 3., alpha);
        lm.lambda = lambda * scaleFactor;
        lm.ni = 2;
        lm.currentChi = tempChi;
        lm.acceptedChi = tempChi;
        lm.cur = 1 - lm.cur;   // accept: discardTop
    } else {
        lm.lambda = lambda * lm.ni;   // reject: pop
        lm.ni *= 2;
    }
    lm.qmax++;
    lm.trials++;
    if (rho < 0 && lm.qmax < 10) return;   // another trial of this iteration
    lm.its++;
    bool term = false;
    if (lm.qmax == 10 || rho == 0) term = true;
    else {
        if ((lm.iniChi - lm.currentChi) * 1e3 < lm.iniChi) lm.nBad++;
        else lm.nBad = 0;
        if (lm.nBad >= 3) term = true;
    }
    if (term || lm.its >= lm.iterations) lm.done = 1;
    else {
        lm.need_lin = 1;
        lm.sys_ready = 0;   // the next iteration linearises at the accepted state
    }
}

template <int PWT>
#ifdef MAM_POINT_SYS_WAVES   // (experiment: a waves-per-SIMD target for k_point_sys, 209 VGPRs = 2 waves by default)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MAM_POINT_SYS_WAVES))) void k_point_sys(
    const Prob* __restrict__ probs) {
#else
__global__ __launch_bounds__(64) void k_point_sys(const Prob* __restrict__ probs) {
#endif
    const Prob& d = probs[blockIdx.y];
    point_sys_body<PWT>(d, lm_head(d.lm));
}

// grid (ceil(L / PW), Q) x 64, after the factorization and its pose epilogue (the trial poses): per point (lanes < PW)
// the back-substitution x_l = D^-1 (b_l - H_pl^T x_p) in edge order (k_backsub_update's; skipped after a failed
// factorization, which leaves the old x), the trial point X + x_l and its computeScale terms x_l (lambda x_l + b_l);
// per slot the trial error of its edge at the trial pose and point (k_linearize's trial pass), summed per wave into
// the chi2 partial of the trial
template <int PWT>
__global__ __launch_bounds__(64) void k_point_trial(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    const LMHead hd = lm_head(d.lm);
    if (hd.status || hd.done) return;
    const int nbp = (d.L + PWT - 1) / PWT;
    if ((int)blockIdx.x >= nbp) return;
    const int lane = threadIdx.x;
    const double lambda = trial_lambda(hd);
    const double* pts = d.pt[hd.cur];
    double* pt_out = d.pt[1 - hd.cur];
    const double* pose_out = d.pose[1 - hd.cur];
    const int h0 = blockIdx.x * PWT, h1 = min(d.L, h0 + PWT);
    __shared__ double xn[PWT * 3];
    // the trial-error pass's slot edge, its pose and that pose's trial value loaded before the back-substitution (one
    // 64-slot chunk, a window's points): their round trips overlap it instead of following the barrier
    const int s0 = d.pe_off[h0], s1 = d.pe_off[h1];
    const bool one = s1 - s0 <= 64;
    int e_pf = 0, ip_pf = 0, pt_pf = h0;
    double T_pf[7];
    if (one && s0 + lane < s1) {
        e_pf = d.pe_idx[s0 + lane];
        ip_pf = d.edge_pose[e_pf];
        pt_pf = d.edge_point[e_pf];
#pragma unroll
        for (int k = 0; k < 7; k++) T_pf[k] = pose_out[7 * (size_t)ip_pf + k];
    }
    double sc = 0.0;
    const int i = h0 + lane;
    // one slot chunk: every slot's H_pl^T x_p term by its own lane (one round of loads for the chunk instead of a
    // dependent walk over the point's slots by the point's lane), summed per point in slot order from LDS
    __shared__ double cst[64 * 3];
    if (one && !hd.fail) {
        double c[3] = {0.0, 0.0, 0.0};
        if (s0 + lane < s1) {
            const int hp = d.slot_hp[s0 + lane];
            if (hp >= 0) {
                const double* B = d.hpl + 18 * (size_t)e_pf;
                const double* xp = d.x + 6 * (size_t)hp;
                double bv[18], xv6[6];
#pragma unroll
                for (int k = 0; k < 18; k++) bv[k] = B[k];
#pragma unroll
                for (int k = 0; k < 6; k++) xv6[k] = xp[k];
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    double v = bv[j] * xv6[0];
#pragma unroll
                    for (int k = 1; k < 6; k++) v += bv[3 * k + j] * xv6[k];
                    c[j] = v;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 3; j++) cst[3 * lane + j] = c[j];
        __syncthreads();
    }
    if (lane < PWT && i < h1) {
        double* xl = d.x + 6 * (size_t)d.Np + 3 * (size_t)i;
        const double* bgl = d.b + 6 * (size_t)d.Np + 3 * (size_t)i;
        double xv[3];
        if (!hd.fail && one) {
            double cl[3];
            for (int k = 0; k < 3; k++) cl[k] = bgl[k];
            const int sa = d.pe_off[i], sz = d.pe_off[i + 1];
            for (int sb = sa; sb < sz; sb++)
#pragma unroll
                for (int j = 0; j < 3; j++) cl[j] -= cst[3 * (sb - s0) + j];
            const double* Di = d.Dinv + 9 * (size_t)i;
            for (int k = 0; k < 3; k++) xv[k] = Di[3 * k] * cl[0] + Di[3 * k + 1] * cl[1] + Di[3 * k + 2] * cl[2];
            for (int k = 0; k < 3; k++) xl[k] = xv[k];
        } else if (!hd.fail) {
            double cl[3];
            for (int k = 0; k < 3; k++) cl[k] = bgl[k];
            const int s1 = d.pe_off[i + 1];
            for (int sb = d.pe_off[i]; sb < s1; sb += PT_PF) {
                int hps[PT_PF], pis[PT_PF];
#pragma unroll
                for (int u = 0; u < PT_PF; u++) {
                    hps[u] = sb + u < s1 ? d.slot_hp[sb + u] : -2;
                    pis[u] = sb + u < s1 ? d.pe_idx[sb + u] : 0;
                }
#pragma unroll
                for (int u = 0; u < PT_PF; u++) {
                    if (hps[u] == -2) break;
                    if (hps[u] < 0) continue;
                    const double* B = d.hpl + 18 * (size_t)pis[u];
                    const double* xp = d.x + 6 * (size_t)hps[u];
#pragma unroll
                    for (int j = 0; j < 3; j++)
#pragma unroll
                        for (int k = 0; k < 6; k++) cl[j] -= B[3 * k + j] * xp[k];
                }
            }
            const double* Di = d.Dinv + 9 * (size_t)i;
            for (int k = 0; k < 3; k++) xv[k] = Di[3 * k] * cl[0] + Di[3 * k + 1] * cl[1] + Di[3 * k + 2] * cl[2];
            for (int k = 0; k < 3; k++) xl[k] = xv[k];
        } else {
            for (int k = 0; k < 3; k++) xv[k] = xl[k];
        }
        for (int k = 0; k < 3; k++) {
            const double X = pts[3 * (size_t)i + k] + xv[k];
            pt_out[3 * (size_t)i + k] = X;
            xn[3 * lane + k] = X;
            sc += xv[k] * (lambda * xv[k] + bgl[k]);
        }
    }
    __syncthreads();
    double r = 0.0;
    if (one) {
        if (s0 + lane < s1) {
            double jr[21], hr[18];
            r = linearize_edge_at(d, T_pf, xn + 3 * (pt_pf - h0), ip_pf, e_pf, false, true, jr, hr);
        }
    } else {
        for (int c0 = s0; c0 < s1; c0 += 64) {
            const int s = c0 + lane;
            if (s < s1) {
                const int e = d.pe_idx[s];
                const int ipose = d.edge_pose[e];
                double jr[21], hr[18];
                r += linearize_edge_at(d, pose_out + 7 * (size_t)ipose, xn + 3 * (d.edge_point[e] - h0), ipose, e, false,
                                       true, jr, hr);
            }
        }
    }
    r = wave_sum_d(r);
    sc = wave_sum_d(sc);
    if (lane == 0) {
        d.part[blockIdx.x] = r;
        d.part_s[blockIdx.x] = sc;
    }
}

// The factorization's epilogue: the trial poses (k_backsub_update's pose part: T <- exp(x_p) T for optimised poses,
// fixed poses copied) and computeScale's pose terms x_p (lambda x_p + b_p) into lm.scale_p (fixed-order block sum),
// by the whole workgroup; xp: the solution's pose part (LDS after a solve; d.x — the previous trial's — after a failed
// factorization, as the reference's update applies the old x)
template <int T>
__device__ __forceinline__ void pose_epilogue(const Prob& d, LM& lm, int cur, const double* xp, double lambda) {
    __shared__ double red[T / 64];
    const int t = threadIdx.x;
    const double* pose = d.pose[cur];
    double* pose_out = d.pose[1 - cur];
    for (int i = t; i < d.P; i += T) {
        const double* Tp = pose + 7 * (size_t)i;
        double* O = pose_out + 7 * (size_t)i;
        const int h = d.pose_h[i];
        if (h < 0) {
            for (int k = 0; k < 7; k++) O[k] = Tp[k];
        } else {
            double u[6];
            for (int k = 0; k < 6; k++) u[k] = xp[6 * h + k];
            se3_exp_mul(u, Tp, O);
        }
    }
    double acc = 0.0;
    for (int j = t; j < 6 * d.Np; j += T) acc += xp[j] * (lambda * xp[j] + d.b[j]);
    acc = wave_sum_d(acc);
    if ((t & 63) == 0) red[t >> 6] = acc;
    __syncthreads();
    if (t == 0) {
        double sum = 0.0;
        for (int w = 0; w < T / 64; w++) sum += red[w];
        lm.scale_p = sum;
    }
}

// ---- the factorization with S's tiles in registers: the form for a dense reduced system (a covisibility window whose
// local keyframes all share MapPoints: every tile of L non-zero, more than the LDS pool holds). The lower-triangle
// tiles (i, j) are numbered by block column from the last and dealt round-robin over the 8 waves (tile q to wave q mod
// 8, register slot q / 8: REG_RT slots of four doubles a lane, the MFMA accumulator layout), the next ones in the LDS
// the launch has left over, the rest (the first columns) in place in S. Blocked
// right-looking LDL^T as ldlt_global computes it, with no global memory round trip inside the loop: per block column
// k (a) the owners stage the diagonal tile and the panel tiles in LDS, (b) wave 0 factors the diagonal tile and
// solves y_k, (c) every thread one panel row (L21 = A21 L11^-T D^-1, y2 -= L21 y1), (d) the owners take their L
// tiles back and update their trailing tiles by f64 MFMA (operands from the staged panel). Then y /= D and the
// backward substitution by block rows: wave 0 solves the diagonal block, each tile of the row subtracts L^T y_k from
// its column's y block (one tile per y block per step: no two writers).
// REG_T threads, REG_RT tiles a wave (at 256 threads a wave may hold 512 registers, but the compiler keeps ~2 registers
// per tile element: 24 tiles a wave at 256 threads, 16 at 512, the same 128 tiles a workgroup without spills)
#ifndef MAM_LBA_REG_T
#define MAM_LBA_REG_T 512
#endif
#ifndef MAM_LBA_REG_RT
#define MAM_LBA_REG_RT 16
#endif
constexpr int REG_T = MAM_LBA_REG_T, REG_RT = MAM_LBA_REG_RT;
#ifndef MAM_REG_PANEL_MFMA
#define MAM_REG_PANEL_MFMA 0   // the panel by L11^-T D^-1 and f64 MFMA (spills at REG_RT 16; 0: per-row forward
                               // substitution)
#endif
__host__ __device__ inline size_t ldlt_reg_lds_bytes(int nt) {
    const int ntri = nt * (nt + 1) / 2, N = 16 * nt;
    return ((size_t)16 * (N - 16) + 2 * (size_t)N + 512) * sizeof(double) + 2 * (size_t)ntri + 16;
}

#ifdef MAM_REG_PROFILE
// cycles per phase summed over workgroups (thread 0 after each barrier): init, (a) staging, (b) diagonal tile,
// (c) panel rows, (d) updates, backward solve, -, WGs
__device__ unsigned long long g_rprof[8];
#define RPROF(k)                                                                     \
    do {                                                                             \
        if (t == 0) {                                                                \
            const long long tn = clock64();                                          \
            atomicAdd(&g_rprof[k], (unsigned long long)(tn - rp0));                  \
            rp0 = tn;                                                                \
        }                                                                            \
    } while (0)
#else
#define RPROF(k) \
    do {         \
    } while (0)
#endif

__device__ __forceinline__ void ldlt_reg(const Prob& d, double* lds, size_t lds_bytes, LdltShared& sh) {
#ifdef MAM_REG_PROFILE
    long long rp0 = clock64();
    if (threadIdx.x == 0) atomicAdd(&g_rprof[7], 1ull);
#endif
    LM& lm = *d.lm;
    constexpr int T = REG_T, NW = T / 64;
    const int nt = d.nt, N = d.npad, n = 6 * d.Np;
    const int ntri = nt * (nt + 1) / 2, nreg = NW * REG_RT;
    const int over = ntri > nreg ? ntri - nreg : 0;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int col = lane & 15, rq = lane >> 4;
    const int mmax = N - 16;
    double* PT = lds;                        // the staged panel, transposed: L(16 (k + 1) + r, 16 k + c) at c * m + r
    double* Y = PT + (size_t)16 * mmax;
    double* Dd = Y + N;                      // D
    double* DB = Dd + N;                     // the diagonal tile: column-major (forward), row-major L (backward)
    double* MB = DB + 256;                   // L11^-T D^-1 (row kk, column j at kk * 16 + j): the panel's right factor
    int8_t* ti = reinterpret_cast<int8_t*>(MB + 256);
    int8_t* tj = ti + ntri;
    uint8_t* tm = reinterpret_cast<uint8_t*>(sh.map);   // the tile mask of L (S + fill)
    gdouble* A = (gdouble*)d.S;
    // overflow tile q: LDS slot q - nreg while they last (after the tables), else in place in S
    double* OT = reinterpret_cast<double*>(((uintptr_t)(tj + ntri) + 15) & ~(uintptr_t)15);
    const size_t used = (size_t)((char*)OT - (char*)lds);
    const int nlds = lds_bytes > used ? (int)((lds_bytes - used) / (256 * sizeof(double))) : 0;
    auto at = [&](int q, int r, int c) -> double* {
        return q - nreg < nlds ? OT + (size_t)(q - nreg) * 256 + r * 16 + c
                               : (double*)(A + (size_t)(16 * ti[q] + r) * N + 16 * tj[q] + c);
    };
    // tile order: by block column from the last (updated at every step) to the first (read once as a panel), so the
    // registers hold the most-updated tiles and the ones in S are a few first columns', touched at a step or two
    for (int q = t; q < ntri; q += T) {
        int r, c;
        tri_index(q, &r, &c);   // r = columns from the end - 1, c = rows below the diagonal
        ti[q] = (int8_t)(nt - 1 - r + c);
        tj[q] = (int8_t)(nt - 1 - r);
    }
    for (int q = t; q < nt * nt; q += T) tm[q] = d.tmask[q];
    for (int i = t; i < N; i += T) Y[i] = i < n ? d.bs[i] : 0.0;
    if (t == 0) sh.fail = 0;
    __syncthreads();
    // S's lower triangle; the padding rows / columns an identity block (as ldlt_global sets it), a diagonal tile's
    // upper triangle zero
    auto s_at = [&](int row, int cc) -> double {
        if (cc > row) return 0.0;
        if (row >= n || cc >= n) return row == cc ? 1.0 : 0.0;
        return A[(size_t)row * N + cc];
    };
    // (the overflow tiles' elements are read and rewritten by the same thread)
    dbl4 R[REG_RT];
#pragma unroll
    for (int u = 0; u < REG_RT; u++) {
        const int q = u * NW + wid;
        R[u] = dbl4{0.0, 0.0, 0.0, 0.0};
        if (q < ntri) {
            const int i = ti[q], j = tj[q];
            if (tm[i * nt + j]) {
#pragma unroll
                for (int r = 0; r < 4; r++) R[u][r] = s_at(16 * i + rq + 4 * r, 16 * j + col);
            }
        }
    }
    for (int x = t; x < over * 256; x += T) {
        const int q = nreg + x / 256, e = x % 256, i = ti[q], j = tj[q];
        const double v = tm[i * nt + j] ? s_at(16 * i + e / 16, 16 * j + e % 16) : 0.0;
        *at(q, e / 16, e % 16) = v;
    }
    __syncthreads();
    RPROF(0);
    for (int k = 0; k < nt; k++) {
        const int m = 16 * (nt - k - 1);
        // (a) the diagonal tile -> DB, the column's panel tiles -> PT
#pragma unroll
        for (int u = 0; u < REG_RT; u++) {
            const int q = u * NW + wid;
            if (q >= ntri) continue;
            const int i = ti[q], j = tj[q];
            if (j != k) continue;
            if (i == k) {
#pragma unroll
                for (int r = 0; r < 4; r++) DB[col * 16 + rq + 4 * r] = R[u][r];
            } else if (tm[i * nt + k]) {
#pragma unroll
                for (int r = 0; r < 4; r++) PT[col * m + 16 * (i - k - 1) + rq + 4 * r] = R[u][r];
            }
        }
        // column k's tiles are q in [c0, c0 + nt - k) (diagonal first), its overflow ones the part past nreg
        const int c0 = (nt - k) * (nt - k - 1) / 2, oq0 = max(c0, nreg), oq1 = c0 + nt - k;
        for (int x = t; x < (oq1 - oq0) * 256; x += T) {
            const int q = oq0 + x / 256, i = k + (q - c0), e = x % 256;
            if (i == k) DB[(e % 16) * 16 + e / 16] = *at(q, e / 16, e % 16);
            else if (tm[i * nt + k]) PT[(e % 16) * m + 16 * (i - k - 1) + e / 16] = *at(q, e / 16, e % 16);
        }
        __syncthreads();
        RPROF(1);
        // (b) wave 0: LDL^T of the diagonal tile, the forward block solve of y_k
        if (wid == 0) {
            double row[NB];
#pragma unroll
            for (int c = 0; c < NB; c++) row[c] = lane < NB ? DB[c * 16 + lane] : 0.0;
            const double dmine = diag16_factor(row, lane);
            const double yv = diag16_forward(row, lane < NB ? Y[16 * k + lane] : 0.0, lane);
            if (lane < NB) {
#pragma unroll
                for (int c = 0; c < NB; c++) sh.Ld[lane * NB + c] = row[c];
                sh.dk[0][lane] = dmine;
                sh.invdk[lane] = dmine != 0.0 ? 1.0 / dmine : 0.0;
                Dd[16 * k + lane] = dmine;
                Y[16 * k + lane] = yv;
                if (dmine == 0.0) sh.fail = 1;
            }
#if MAM_REG_PANEL_MFMA
            // L11^-1 by 16 forward solves of unit vectors (independent chains, interleaved), then MB = L11^-T D^-1
            // (two halves of 8 columns: the tiles' registers leave room for 8 chains)
            const double invd = dmine != 0.0 ? 1.0 / dmine : 0.0;
#pragma unroll
            for (int h = 0; h < NB; h += 8) {
                double xc[8];
#pragma unroll
                for (int c = 0; c < 8; c++) xc[c] = lane == h + c ? 1.0 : 0.0;
#pragma unroll
                for (int j = 0; j < NB; j++) {
#pragma unroll
                    for (int c = 0; c < 8; c++) {
                        if (h + c > j) continue;   // X(j, c) = 0 for j < c: nothing to subtract
                        const double xj = bcast16_d(xc[c], j);
                        if (lane > j) xc[c] = fma(-row[j], xj, xc[c]);
                    }
                }
                if (lane < NB) {
#pragma unroll
                    for (int c = 0; c < 8; c++) MB[(h + c) * 16 + lane] = xc[c] * invd;   // M(c, lane) = Linv(lane, c) / d
                }
            }
#endif
        }
        __syncthreads();
        RPROF(2);
#if MAM_REG_PANEL_MFMA
        // (c) the panel L21 = A21 M by f64 MFMA, one 16-row tile per wave in place (a wave reads and writes only its
        // tile's rows); y2 -= L21 y1 in (d)
        for (int rt = wid; rt < m / 16; rt += NW) {
            if (!tm[(k + 1 + rt) * nt + k]) continue;
            dbl4 c4 = dbl4{0.0, 0.0, 0.0, 0.0};
            double av[4], bv[4];
#pragma unroll
            for (int k0 = 0; k0 < NB; k0 += 4) {
                av[k0 / 4] = PT[(k0 + rq) * m + 16 * rt + col];
                bv[k0 / 4] = MB[(k0 + rq) * 16 + col];
            }
#pragma unroll
            for (int k0 = 0; k0 < 4; k0++) c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[k0], bv[k0], c4, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; r++) PT[col * m + 16 * rt + rq + 4 * r] = c4[r];
        }
        __syncthreads();
        RPROF(3);
        for (int r = t; r < m; r += T) {
            const int i = 16 * (k + 1) + r;
            if (!tm[(i >> 4) * nt + k]) continue;
            double yi = Y[i];
#pragma unroll
            for (int j = 0; j < NB; j++) yi = fma(-PT[j * m + r], Y[16 * k + j], yi);
            Y[i] = yi;
        }
#else
        // (c) the panel rows in place: L21 = A21 L11^-T D^-1, y2 -= L21 y1
        for (int r = t; r < m; r += T) {
            const int i = 16 * (k + 1) + r;
            if (!tm[(i >> 4) * nt + k]) continue;
            asm volatile("" ::: "memory");
            double w[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) w[j] = PT[j * m + r];
#pragma unroll
            for (int j = 1; j < NB; j++) {
#pragma unroll
                for (int kk = 0; kk < j; kk++) w[j] = fma(-w[kk], sh.Ld[j * NB + kk], w[j]);
            }
            double yi = Y[i];
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const double lij = w[j] * sh.invdk[j];
                PT[j * m + r] = lij;
                yi = fma(-lij, Y[16 * k + j], yi);
            }
            Y[i] = yi;
        }
        __syncthreads();
        RPROF(3);
#endif
        // (d) the column's L back into its tiles; the trailing tiles -= L(i, k) D L(j, k)^T
#pragma unroll
        for (int u = 0; u < REG_RT; u++) {
            const int q = u * NW + wid;
            if (q >= ntri) continue;
            const int i = ti[q], j = tj[q];
            if (j == k) {
                if (i == k) {
#pragma unroll
                    for (int r = 0; r < 4; r++) R[u][r] = sh.Ld[(rq + 4 * r) * NB + col];
                } else if (tm[i * nt + k]) {
#pragma unroll
                    for (int r = 0; r < 4; r++) R[u][r] = PT[col * m + 16 * (i - k - 1) + rq + 4 * r];
                }
            } else if (j > k && tm[i * nt + j] && tm[i * nt + k] && tm[j * nt + k]) {
                const int bi = 16 * (i - k - 1), bj = 16 * (j - k - 1);
#pragma unroll
                for (int k0 = 0; k0 < NB; k0 += 4) {
                    const int kk = k0 + rq;
                    const double av = -PT[kk * m + bi + col];
                    const double bv = PT[kk * m + bj + col] * sh.dk[0][kk];
                    R[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, R[u], 0, 0, 0);
                }
            }
        }
        for (int q = nreg + wid; q < c0 + nt - k; q += NW) {   // (columns < k are final)
            const int i = ti[q], j = tj[q];
            if (j == k) {
                if (i == k) {
#pragma unroll
                    for (int r = 0; r < 4; r++) *at(q, rq + 4 * r, col) = sh.Ld[(rq + 4 * r) * NB + col];
                } else if (tm[i * nt + k]) {
#pragma unroll
                    for (int r = 0; r < 4; r++) *at(q, rq + 4 * r, col) = PT[col * m + 16 * (i - k - 1) + rq + 4 * r];
                }
            } else if (j > k && tm[i * nt + j] && tm[i * nt + k] && tm[j * nt + k]) {
                const int bi = 16 * (i - k - 1), bj = 16 * (j - k - 1);
                dbl4 c4;
#pragma unroll
                for (int r = 0; r < 4; r++) c4[r] = *at(q, rq + 4 * r, col);
#pragma unroll
                for (int k0 = 0; k0 < NB; k0 += 4) {
                    const int kk = k0 + rq;
                    const double av = -PT[kk * m + bi + col];
                    const double bv = PT[kk * m + bj + col] * sh.dk[0][kk];
                    c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c4, 0, 0, 0);
                }
#pragma unroll
                for (int r = 0; r < 4; r++) *at(q, rq + 4 * r, col) = c4[r];
            }
        }
        __syncthreads();
        RPROF(4);
    }
    if (t == 0) lm.fail = sh.fail;
    if (sh.fail) return;   // uniform (LDS flag after the last barrier)
    for (int i = t; i < N; i += T) Y[i] /= Dd[i];
    __syncthreads();
    // backward substitution L^T x = y by block rows, the last first
    for (int k = nt - 1; k >= 0; k--) {
        const int qd = (nt - k) * (nt - k - 1) / 2;   // the diagonal tile (row-major L into DB)
        if (qd < nreg) {
            if (qd % NW == wid) {
#pragma unroll
                for (int u = 0; u < REG_RT; u++)
                    if (u * NW + wid == qd) {
#pragma unroll
                        for (int r = 0; r < 4; r++) DB[(rq + 4 * r) * 16 + col] = R[u][r];
                    }
            }
        } else {
            for (int x = t; x < 256; x += T) DB[x] = *at(qd, x / 16, x % 16);
        }
        __syncthreads();
        if (wid == 0) {
            double cl[NB];   // lane c: L(kb + j, kb + c)
#pragma unroll
            for (int j = 0; j < NB; j++) cl[j] = lane < NB ? DB[j * 16 + lane] : 0.0;
            double v = lane < NB ? Y[16 * k + lane] : 0.0;
#pragma unroll
            for (int j = NB - 1; j >= 0; j--) {
                const double xj = bcast16_d(v, j);
                if (lane < j) v = fma(-cl[j], xj, v);
            }
            if (lane < NB) Y[16 * k + lane] = v;
        }
        __syncthreads();
        // y_j -= L(k, j)^T y_k for the row's non-zero tiles j < k
        const double y0 = Y[16 * k + rq], y1 = Y[16 * k + rq + 4], y2 = Y[16 * k + rq + 8], y3 = Y[16 * k + rq + 12];
#pragma unroll
        for (int u = 0; u < REG_RT; u++) {
            const int q = u * NW + wid;
            if (q >= ntri) continue;
            const int i = ti[q], j = tj[q];
            if (i != k || j >= k || !tm[i * nt + j]) continue;
            double p = R[u][0] * y0;
            p = fma(R[u][1], y1, p);
            p = fma(R[u][2], y2, p);
            p = fma(R[u][3], y3, p);
            p += __shfl_xor(p, 16, 64);
            p += __shfl_xor(p, 32, 64);
            if (rq == 0) Y[16 * j + col] -= p;
        }
        for (int j = wid; j < k; j += NW) {   // row k's tiles (k, j): q = (nt - j)(nt - j - 1) / 2 + k - j
            const int q = (nt - j) * (nt - j - 1) / 2 + k - j;
            if (q < nreg || !tm[k * nt + j]) continue;
            double p = *at(q, rq, col) * y0;
            p = fma(*at(q, rq + 4, col), y1, p);
            p = fma(*at(q, rq + 8, col), y2, p);
            p = fma(*at(q, rq + 12, col), y3, p);
            p += __shfl_xor(p, 16, 64);
            p += __shfl_xor(p, 32, 64);
            if (rq == 0) Y[16 * j + col] -= p;
        }
        __syncthreads();
    }
    for (int i = t; i < n; i += T) d.x[6 * (size_t)d.iperm[i / 6] + i % 6] = Y[i];   // (pose order)
    RPROF(5);
}

// grid (Q) x LDLT_THREADS: the register form for the problems it takes (dense, nt <= reg_nt_max; k_ldlt_any leaves
// them alone), then the trial poses
__global__ __launch_bounds__(REG_T) void k_ldlt_reg(const Prob* __restrict__ probs, int reg_nt_max,
                                                           size_t lds_bytes) {
    extern __shared__ __attribute__((aligned(16))) double lds_dyn[];
    __shared__ LdltShared sh;
    const Prob& d = probs[blockIdx.x];
    const LMHead hd = lm_head(d.lm);
    if (hd.status || hd.done) return;
    if (d.Np == 0 || hd.tiles_lds || d.nt > reg_nt_max) return;
    ldlt_reg(d, lds_dyn, lds_bytes, sh);
    __syncthreads();
    pose_epilogue<REG_T>(d, *d.lm, hd.cur, d.x, trial_lambda(hd));
}

// ---- the dense factorization over several workgroups per problem (the column-chain form): a dense reduced system
// (the covisibility windows of a map where every local keyframe shares MapPoints with every other: ~300-380 unknowns,
// no zero tile) is ~10-18 MFLOP, too much dependent work for the one CU of the single-workgroup forms (~425 us a
// launch of 16 such windows). Here MW_G workgroups per problem claim block columns in order from a per-problem counter
// and each runs its column's whole left-looking chain: the column's tiles in registers (wave w: row blocks j + w,
// j + w + 8, ...), then for every k < j with L(j, k) != 0: wait for column k's flag, L(i, k) D_k L(j, k)^T off its tiles
// by f64 MFMA (the same products in the same k order as the right-looking forms) and y_j -= L(j, k) y_k; then its own
// panel: the diagonal tile's LDL^T on wave 0, L21 = A21 L11^-T D^-1 one row a thread, L(:, j), D_j and the solved y_j
// stored, the flag raised. The workgroup that finishes the last column does the backward substitution (row by row,
// the next row's tiles loaded before the diagonal solve) and the trial poses. Deadlock-free without co-residency:
// a column waits only for smaller columns, claimed earlier by running workgroups (one resident workgroup alone runs
// every column in turn). Cross-workgroup data (L, D, y, flags) moves by agent-scope relaxed atomics (sc1 loads /
// stores, coherent across XCDs) and an s_waitcnt before the flag — no L2 write-back / invalidate per step (an
// agent-scope release writes the whole L2 back: DESIGN §6). Flags carry the launch's tag (base + 1; base advances by
// the claims a launch makes), so nothing is reset between launches.
#ifndef MAM_LBA_MW_G
#define MAM_LBA_MW_G 8   // workgroups per dense problem
#endif
#ifndef MAM_LBA_MW_T
#define MAM_LBA_MW_T 256   // threads: one wave per SIMD, 512 registers a wave (the column's tiles + the panel rows)
#endif
constexpr int MW_G = MAM_LBA_MW_G, MW_NT_MAX = 40, MW_T = MAM_LBA_MW_T;
__host__ __device__ inline size_t ldlt_mw_lds_bytes(int npad) {
    return ((size_t)16 * (npad > 16 ? npad - 16 : 0) + 256 + 256 + 80) * sizeof(double);
}
// (global address space: flat accesses would also count in lgkmcnt)
typedef __attribute__((address_space(1))) int gint;
__device__ __forceinline__ double ld_c(const double* p) {
    return __hip_atomic_load((gdouble*)const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_c(double* p, double v) {
    __hip_atomic_store((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_ci(const int* p) {
    return __hip_atomic_load((gint*)const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ci(int* p, int v) {
    __hip_atomic_store((gint*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The published data (L, D, y, a helper's partial column) is read after the flag with agent-coherent loads too:
// plain loads after an L1 invalidate failed the parity tests on the lookahead form (a workgroup's L2 can hold a line
// another XCD's workgroup rewrote since: a helper's copy of the partial column it published, read back as the panel's
// final L by a later helper on that XCD). MAM_MW_SC1_LOADS=0 keeps the plain loads for the experiment.
#ifndef MAM_MW_SC1_LOADS
#define MAM_MW_SC1_LOADS 1
#endif
__device__ __forceinline__ double ld_pub(const double* p) {
#if MAM_MW_SC1_LOADS
    return ld_c(p);
#else
    return *(const gdouble*)p;
#endif
}
__device__ __forceinline__ void inv_l1() {
#if !MAM_MW_SC1_LOADS
    asm volatile("buffer_inv sc0" ::: "memory");
#endif
}
// thread 0 waits for column k's flag (bounded: a wait that never ends marks the factorization failed instead of hanging)
__device__ __forceinline__ void mw_wait(int* mw, int k, int tag) {
    int it = 0;
    while (ld_ci(&mw[8 + k]) != tag) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > (1 << 20)) {
            st_ci(&mw[2], 2);
            break;
        }
    }
}

// returns true in the workgroup that finished the factorization and wrote d.x (it runs the pose epilogue)
#ifdef MAM_MW_PROFILE
// cycles summed over workgroups (thread 0): flag waits, the k steps' loads + updates, the panel, the publish, the
// backward pass; [6] columns, [7] k steps
__device__ unsigned long long g_mwprof[8];
#define MWPROF(k)                                                                    \
    do {                                                                             \
        if (t == 0) {                                                                \
            const long long tn = clock64();                                          \
            atomicAdd(&g_mwprof[k], (unsigned long long)(tn - mp0));                 \
            mp0 = tn;                                                                \
        }                                                                            \
    } while (0)
#else
#define MWPROF(k) \
    do {          \
    } while (0)
#endif
template <int T>
__device__ bool ldlt_mw(const Prob& d, double* lds, LdltShared& sh, int G) {
#ifdef MAM_MW_PROFILE
    long long mp0 = clock64();
#endif
    constexpr int NW = T / 64, RT = (MW_NT_MAX + NW - 1) / NW;   // tiles a wave holds
    const int nt = d.nt, N = d.npad, n = 6 * d.Np;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6, col = lane & 15, rq = lane >> 4;
    int* mw = d.mw;
    double* S = d.S;
    double* Yg = d.ws;
    double* Dg = d.ws + N;
    double* PT = lds;                         // the panel, transposed (c * m + r); the backward pass's z
    double* DB = PT + (size_t)16 * (N - 16);  // the diagonal tile, column-major
    double* LJ = DB + 256;                    // L(j, k), row-major
    double* DK = LJ + 256;                    // D_k, then D_j
    double* YK = DK + 16;                     // y_k
    double* YJ = YK + 16;                     // the column's y block
    uint8_t* tm = reinterpret_cast<uint8_t*>(sh.map);
    __shared__ int s_col;
    for (int q = t; q < nt * nt; q += T) tm[q] = ((const __attribute__((address_space(1))) uint8_t*)d.tmask)[q];
    const int base = ld_ci(&mw[1]), tag = base + 1;
    auto s_at = [&](int row, int cc) -> double {
        if (cc > row) return 0.0;
        if (row >= n || cc >= n) return row == cc ? 1.0 : 0.0;
        return S[(size_t)row * N + cc];
    };
    bool last = false;
    for (;;) {
        __syncthreads();
        if (t == 0) s_col = atomicAdd(&mw[0], 1) - base;
        __syncthreads();
        const int j = s_col;
        if (j >= nt) {
            if (t == 0 && j == nt + G - 1) st_ci(&mw[1], base + nt + G);   // every workgroup has read base
            break;
        }
        // the column's tiles (S as k_schur_blk wrote it: padding identity, the diagonal tile's upper triangle zero)
        dbl4 R[RT];
#pragma unroll
        for (int u = 0; u < RT; u++) {
            const int i = j + wid + NW * u;
            R[u] = dbl4{0.0, 0.0, 0.0, 0.0};
            if (i < nt && tm[i * nt + j]) {
#pragma unroll
                for (int r = 0; r < 4; r++) R[u][r] = s_at(16 * i + rq + 4 * r, 16 * j + col);
            }
        }
        if (t < 16) YJ[t] = 16 * j + t < n ? d.bs[16 * j + t] : 0.0;
        for (int k = 0; k < j; k++) {
            if (!tm[j * nt + k]) continue;
            __syncthreads();   // (the previous step's LJ / YK reads)
            MWPROF(1);
            if (t == 0) mw_wait(mw, k, tag);
            __syncthreads();
            inv_l1();
            MWPROF(0);
#ifdef MAM_MW_PROFILE
            if (t == 0) atomicAdd(&g_mwprof[7], 1ull);
#endif
            // L(j, k), D_k, y_k and the wave's A operands L(i, k) requested together: one memory round trip
            static_assert(T == 256, "one L(j, k) element a thread");
            const double ljv = ld_pub(&S[(size_t)(16 * j + t / 16) * N + 16 * k + t % 16]);
            double dkv = 0.0, ykv = 0.0;
            if (t < 16) {
                dkv = ld_pub(&Dg[16 * k + t]);
                ykv = ld_pub(&Yg[16 * k + t]);
            }
            double av[RT][4];
#pragma unroll
            for (int u = 0; u < RT; u++) {
                const int i = j + wid + NW * u;
                const bool on = i < nt && tm[i * nt + k];
#pragma unroll
                for (int q4 = 0; q4 < 4; q4++)
                    av[u][q4] = on ? -ld_pub(&S[(size_t)(16 * i + col) * N + 16 * k + 4 * q4 + rq]) : 0.0;
            }
            LJ[t] = ljv;
            if (t < 16) {
                DK[t] = dkv;
                YK[t] = ykv;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < RT; u++) {
                const int i = j + wid + NW * u;
                if (i >= nt || !tm[i * nt + k]) continue;
#pragma unroll
                for (int q4 = 0; q4 < 4; q4++) {
                    const int kk = 4 * q4 + rq;
                    R[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u][q4], LJ[col * 16 + kk] * DK[kk], R[u], 0, 0, 0);
                }
            }
            if (t < 16) {
                double v = YJ[t];
#pragma unroll
                for (int c = 0; c < NB; c++) v = fma(-LJ[t * 16 + c], YK[c], v);
                YJ[t] = v;
            }
        }
        __syncthreads();
        MWPROF(1);
#ifdef MAM_MW_PROFILE
        if (t == 0) atomicAdd(&g_mwprof[6], 1ull);
#endif
        // the column's panel: stage, factor the diagonal tile, the panel rows
        const int m = 16 * (nt - j - 1);
#pragma unroll
        for (int u = 0; u < RT; u++) {
            const int i = j + wid + NW * u;
            if (i >= nt) continue;
            if (i == j) {
#pragma unroll
                for (int r = 0; r < 4; r++) DB[col * 16 + rq + 4 * r] = R[u][r];
            } else if (tm[i * nt + j]) {
#pragma unroll
                for (int r = 0; r < 4; r++) PT[col * m + 16 * (i - j - 1) + rq + 4 * r] = R[u][r];
            }
        }
        __syncthreads();
        if (wid == 0) {
            double row[NB];
#pragma unroll
            for (int c = 0; c < NB; c++) row[c] = lane < NB ? DB[c * 16 + lane] : 0.0;
            const double dmine = diag16_factor(row, lane);
            const double yv = diag16_forward(row, lane < NB ? YJ[lane] : 0.0, lane);
            if (lane < NB) {
#pragma unroll
                for (int c = 0; c < NB; c++) sh.Ld[lane * NB + c] = row[c];
                sh.invdk[lane] = dmine != 0.0 ? 1.0 / dmine : 0.0;
                DK[lane] = dmine;
                YJ[lane] = yv;
                if (dmine == 0.0) st_ci(&mw[2], 1);
            }
        }
        __syncthreads();
        for (int r = t; r < m; r += T) {
            if (!tm[(j + 1 + r / 16) * nt + j]) continue;
            asm volatile("" ::: "memory");   // (keeps the 120 L11 reads in the loop: hoisted they take 240 VGPRs)
            double w[NB];
#pragma unroll
            for (int c = 0; c < NB; c++) w[c] = PT[c * m + r];
            // right-looking: once w[kk] is final its updates are independent (each w[c] still takes them in kk order:
            // the same operations as the row's dot products, 16 dependent steps instead of 120)
#pragma unroll
            for (int kk = 0; kk < NB - 1; kk++) {
#pragma unroll
                for (int c = kk + 1; c < NB; c++) w[c] = fma(-w[kk], sh.Ld[c * NB + kk], w[c]);
            }
#pragma unroll
            for (int c = 0; c < NB; c++) PT[c * m + r] = w[c] * sh.invdk[c];
        }
        __syncthreads();
        MWPROF(2);
        // publish L(:, j) (the diagonal tile's unit lower part; D_j apart), D_j, y_j; then the flag
        for (int x = t; x < 256; x += T) {
            const int r = x / 16, c = x % 16;
            if (c < r) st_c(&S[(size_t)(16 * j + r) * N + 16 * j + c], sh.Ld[r * NB + c]);
        }
        for (int x = t; x < m * 16; x += T) {
            const int r = x / 16, c = x % 16;
            if (tm[(j + 1 + r / 16) * nt + j]) st_c(&S[(size_t)(16 * (j + 1) + r) * N + 16 * j + c], PT[c * m + r]);
        }
        if (t < 16) {
            st_c(&Dg[16 * j + t], DK[t]);
            st_c(&Yg[16 * j + t], YJ[t]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) st_ci(&mw[8 + j], tag);
        MWPROF(3);
        if (j == nt - 1) last = true;
    }
    if (!last) return false;
    // the backward substitution L^T x = D^-1 y, by block rows from the last (every column's flag first: the last
    // column's chain skipped the columns whose L(nt - 1, k) is zero)
    if (t == 0)
        for (int k = 0; k < nt; k++) mw_wait(mw, k, tag);
    __syncthreads();
    inv_l1();
    LM& lm = *d.lm;
    const int fl = ld_ci(&mw[2]);
    if (t == 0) lm.fail = fl != 0;
    if (fl) return true;
    double* Z = PT;
    for (int i = t; i < N; i += T) Z[i] = ld_pub(&Yg[i]) / ld_pub(&Dg[i]);
    __syncthreads();
    for (int k = nt - 1; k >= 0; k--) {
        // row k's tiles (k, i), i < k, loaded first (their latency under the diagonal solve)
        dbl4 Q[RT];
#pragma unroll
        for (int u = 0; u < RT; u++) {
            const int i = wid + NW * u;
            Q[u] = dbl4{0.0, 0.0, 0.0, 0.0};
            if (i < k && tm[k * nt + i]) {
#pragma unroll
                for (int r = 0; r < 4; r++) Q[u][r] = ld_pub(&S[(size_t)(16 * k + rq + 4 * r) * N + 16 * i + col]);
            }
        }
        if (wid == 0) {
            double cl[NB];   // lane c: L(kb + jj, kb + c)
#pragma unroll
            for (int jj = 0; jj < NB; jj++)
                cl[jj] = (lane < NB && jj > lane) ? ld_pub(&S[(size_t)(16 * k + jj) * N + 16 * k + lane]) : 0.0;
            double v = lane < NB ? Z[16 * k + lane] : 0.0;
#pragma unroll
            for (int jj = NB - 1; jj >= 0; jj--) {
                const double xj = bcast16_d(v, jj);
                if (lane < jj) v = fma(-cl[jj], xj, v);
            }
            if (lane < NB) Z[16 * k + lane] = v;
        }
        __syncthreads();
        const double y0 = Z[16 * k + rq], y1 = Z[16 * k + rq + 4], y2 = Z[16 * k + rq + 8], y3 = Z[16 * k + rq + 12];
#pragma unroll
        for (int u = 0; u < RT; u++) {
            const int i = wid + NW * u;
            if (i >= k || !tm[k * nt + i]) continue;
            double p = Q[u][0] * y0;
            p = fma(Q[u][1], y1, p);
            p = fma(Q[u][2], y2, p);
            p = fma(Q[u][3], y3, p);
            p += __shfl_xor(p, 16, 64);
            p += __shfl_xor(p, 32, 64);
            if (rq == 0) Z[16 * i + col] -= p;
        }
        __syncthreads();
    }
    for (int i = t; i < n; i += T) d.x[6 * (size_t)d.iperm[i / 6] + i % 6] = Z[i];   // (pose order)
    MWPROF(4);
    return true;
}

// grid (Q) x LDLT_THREADS: either form per problem (k_struct_tiles' choice, read on the device), so the host launches
// one factorization per trial without reading the choice back; dynamic LDS: the larger of the two forms' needs
// The lookahead form of the column chain (MAM_MW_LOOKAHEAD=1): the workgroup that claims column 0 becomes the panel
// workgroup and factors every column's panel in turn, applying each column's last update L(i, j-1) D L(j, j-1)^T from
// its own LDS copy of the previous panel (no global round trip on the critical path); the other workgroups claim
// columns in order, apply every earlier update but the last (waiting on the panel flags), publish the column's tiles
// and partial y in place and raise the column's ready flag. The panel workgroup takes a column nobody has claimed yet
// itself (compare-and-swap on the counter), so one resident workgroup alone still runs every column: no co-residency
// needed. Per column on the critical path: the ready column's load, one update, the diagonal tile, the panel rows,
// the publish — ~half the chain form's handoff.
#ifndef MAM_MW_DEFER
#define MAM_MW_DEFER 1   // the panel flag raised after the next column's load and update (its stores drain meanwhile)
#endif
template <int T>
__device__ bool ldlt_mw_la(const Prob& d, double* lds, LdltShared& sh, int G) {
    constexpr int NW = T / 64, RT = (MW_NT_MAX + NW - 1) / NW;
    const int nt = d.nt, N = d.npad, n = 6 * d.Np;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6, col = lane & 15, rq = lane >> 4;
    int* mw = d.mw;
    double* S = d.S;
    double* Yg = d.ws;
    double* Dg = d.ws + N;
    double* PT = lds;                         // the panel, transposed (c * m + r)
    double* DB = PT + (size_t)16 * (N - 16);  // the diagonal tile, column-major
    double* LJ = DB + 256;                    // L(j, k), row-major
    double* DK = LJ + 256;                    // D of the last factored column
    double* YK = DK + 16;                     // y of the last factored column (solved)
    double* YJ = YK + 16;                     // the column's y block
    double* DP = YJ + 16;                     // the panel workgroup's last column: D
    double* YP = DP + 16;                     // and its solved y
    uint8_t* tm = reinterpret_cast<uint8_t*>(sh.map);
    __shared__ int s_col;
    for (int q = t; q < nt * nt; q += T) tm[q] = ((const __attribute__((address_space(1))) uint8_t*)d.tmask)[q];
    const int base = ld_ci(&mw[1]), tag = base + 1;
    auto s_at = [&](int row, int cc) __attribute__((always_inline)) -> double {
        if (cc > row) return 0.0;
        if (row >= n || cc >= n) return row == cc ? 1.0 : 0.0;
        return S[(size_t)row * N + cc];
    };
    dbl4 R[RT];
    // the column's tiles as k_schur_blk wrote S, y_j from bs
    auto load_orig = [&](int j) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < RT; u++) {
            const int i = j + wid + NW * u;
            R[u] = dbl4{0.0, 0.0, 0.0, 0.0};
            if (i < nt && tm[i * nt + j]) {
#pragma unroll
                for (int r = 0; r < 4; r++) R[u][r] = s_at(16 * i + rq + 4 * r, 16 * j + col);
            }
        }
        if (t < 16) YJ[t] = 16 * j + t < n ? d.bs[16 * j + t] : 0.0;
    };
    // L(i, k) D_k L(j, k)^T off the column's tiles and y_j -= L(j, k) y_k for k in [k0, k1), from the published panels
    auto apply_published = [&](int j, int k0, int k1) __attribute__((always_inline)) {
        for (int k = k0; k < k1; k++) {
            if (!tm[j * nt + k]) continue;
            __syncthreads();
            if (t == 0) mw_wait(mw, k, tag);
            __syncthreads();
            inv_l1();
            const double ljv = ld_pub(&S[(size_t)(16 * j + t / 16) * N + 16 * k + t % 16]);
            double dkv = 0.0, ykv = 0.0;
            if (t < 16) {
                dkv = ld_pub(&Dg[16 * k + t]);
                ykv = ld_pub(&Yg[16 * k + t]);
            }
            double av[RT][4];
#pragma unroll
            for (int u = 0; u < RT; u++) {
                const int i = j + wid + NW * u;
                const bool on = i < nt && tm[i * nt + k];
#pragma unroll
                for (int q4 = 0; q4 < 4; q4++)
                    av[u][q4] = on ? -ld_pub(&S[(size_t)(16 * i + col) * N + 16 * k + 4 * q4 + rq]) : 0.0;
            }
            __syncthreads();   // (LJ / DK / YK of the previous step read)
            LJ[t] = ljv;
            if (t < 16) {
                DK[t] = dkv;
                YK[t] = ykv;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < RT; u++) {
                const int i = j + wid + NW * u;
                if (i >= nt || !tm[i * nt + k]) continue;
#pragma unroll
                for (int q4 = 0; q4 < 4; q4++) {
                    const int kk = 4 * q4 + rq;
                    R[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u][q4], LJ[col * 16 + kk] * DK[kk], R[u], 0, 0, 0);
                }
            }
            if (t < 16) {
                double v = YJ[t];
#pragma unroll
                for (int c = 0; c < NB; c++) v = fma(-LJ[t * 16 + c], YK[c], v);
                YJ[t] = v;
            }
        }
        __syncthreads();
    };
    // one loop for both roles (a single site of the chain's updates keeps the register allocation in bounds)
    bool panel = false;
    int jp = 0, mprev = 0, pending = -1;   // (pending: a published panel whose flag waits for its stores, MAM_MW_DEFER)
    for (;;) {
        int j;
        bool own = true;
        if (!panel) {
            __syncthreads();
            if (t == 0) s_col = atomicAdd(&mw[0], 1) - base;
            __syncthreads();
            j = s_col;
            if (j >= nt) {
                if (t == 0 && j == nt + G - 2) st_ci(&mw[1], base + nt + G - 1);   // the helpers' last claim
                return false;
            }
            if (j == 0) panel = true;
        } else {
            j = jp;
            __syncthreads();
            // a ready column is a helper's (one load); else take it if nobody has claimed it
            if (t == 0)
                s_col = ld_ci(&mw[48 + j]) == tag ? 0 : (atomicCAS(&mw[0], base + j, base + j + 1) == base + j ? 1 : 0);
            __syncthreads();
            own = s_col != 0;
        }
        if (own) {   // every update of column j but the last, from the published panels
            load_orig(j);
            apply_published(j, 0, j - 1);
        }
        if (!panel) {   // a helper: the partially updated column published in place, then its ready flag
#pragma unroll
            for (int u = 0; u < RT; u++) {
                const int i = j + wid + NW * u;
                if (i >= nt || !tm[i * nt + j]) continue;
#pragma unroll
                for (int r = 0; r < 4; r++) st_c(&S[(size_t)(16 * i + rq + 4 * r) * N + 16 * j + col], R[u][r]);
            }
            if (t < 16) st_c(&Yg[16 * j + t], YJ[t]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) st_ci(&mw[48 + j], tag);
            continue;
        }
        if (j > 0) {
            if (!own) {   // a helper's column: wait for it, then its tiles and partial y
                if (t == 0) {
                    int it = 0;
                    while (ld_ci(&mw[48 + j]) != tag) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++it > (1 << 20)) {
                            st_ci(&mw[2], 2);
                            break;
                        }
                    }
                }
                __syncthreads();
                inv_l1();
#pragma unroll
                for (int u = 0; u < RT; u++) {
                    const int i = j + wid + NW * u;
                    R[u] = dbl4{0.0, 0.0, 0.0, 0.0};
                    if (i < nt && tm[i * nt + j]) {
#pragma unroll
                        for (int r = 0; r < 4; r++) R[u][r] = ld_pub(&S[(size_t)(16 * i + rq + 4 * r) * N + 16 * j + col]);
                    }
                }
                if (t < 16) YJ[t] = ld_pub(&Yg[16 * j + t]);
            }
            // the last update, from the previous panel still in LDS: L(i, j - 1) at PT[c * mprev + 16 (i - j) + r]
            if (tm[j * nt + j - 1]) {
#pragma unroll
                for (int u = 0; u < RT; u++) {
                    const int i = j + wid + NW * u;
                    if (i >= nt || !tm[i * nt + j - 1]) continue;
#pragma unroll
                    for (int q4 = 0; q4 < 4; q4++) {
                        const int kk = 4 * q4 + rq;
                        R[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(-PT[kk * mprev + 16 * (i - j) + col],
                                                                    PT[kk * mprev + col] * DP[kk], R[u], 0, 0, 0);
                    }
                }
                if (t < 16) {
                    double v = YJ[t];
#pragma unroll
                    for (int cc = 0; cc < NB; cc++) v = fma(-PT[cc * mprev + t], YP[cc], v);
                    YJ[t] = v;
                }
            }
#if MAM_MW_DEFER
            // the previous panel's flag, its stores drained under this column's load and update
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
            __syncthreads();   // (the previous panel read before this one is staged over it)
#if MAM_MW_DEFER
            if (t == 0 && pending >= 0) st_ci(&mw[8 + pending], tag);
            pending = -1;
#endif
        }
        // the panel of column j: stage, the diagonal tile on wave 0, the rows, publish
        const int m = 16 * (nt - j - 1);
#pragma unroll
        for (int u = 0; u < RT; u++) {
            const int i = j + wid + NW * u;
            if (i >= nt) continue;
            if (i == j) {
#pragma unroll
                for (int r = 0; r < 4; r++) DB[col * 16 + rq + 4 * r] = R[u][r];
            } else if (tm[i * nt + j]) {
#pragma unroll
                for (int r = 0; r < 4; r++) PT[col * m + 16 * (i - j - 1) + rq + 4 * r] = R[u][r];
            } else {
#pragma unroll
                for (int r = 0; r < 4; r++) PT[col * m + 16 * (i - j - 1) + rq + 4 * r] = 0.0;
            }
        }
        __syncthreads();
        if (wid == 0) {
            double row[NB];
#pragma unroll
            for (int cc = 0; cc < NB; cc++) row[cc] = lane < NB ? DB[cc * 16 + lane] : 0.0;
            const double dmine = diag16_factor(row, lane);
            const double yv = diag16_forward(row, lane < NB ? YJ[lane] : 0.0, lane);
            if (lane < NB) {
#pragma unroll
                for (int cc = 0; cc < NB; cc++) sh.Ld[lane * NB + cc] = row[cc];
                sh.invdk[lane] = dmine != 0.0 ? 1.0 / dmine : 0.0;
                DP[lane] = dmine;
                YP[lane] = yv;
                if (dmine == 0.0) st_ci(&mw[2], 1);
            }
        }
        __syncthreads();
        for (int r = t; r < m; r += T) {
            if (!tm[(j + 1 + r / 16) * nt + j]) continue;
            double w[NB];
#pragma unroll
            for (int cc = 0; cc < NB; cc++) w[cc] = PT[cc * m + r];
#pragma unroll
            for (int kk = 0; kk < NB - 1; kk++) {
#pragma unroll
                for (int cc = kk + 1; cc < NB; cc++) w[cc] = fma(-w[kk], sh.Ld[cc * NB + kk], w[cc]);
            }
#pragma unroll
            for (int cc = 0; cc < NB; cc++) PT[cc * m + r] = w[cc] * sh.invdk[cc];
        }
        __syncthreads();
        for (int x = t; x < 256; x += T) {
            const int r = x / 16, cc = x % 16;
            if (cc < r) st_c(&S[(size_t)(16 * j + r) * N + 16 * j + cc], sh.Ld[r * NB + cc]);
        }
        for (int x = t; x < m * 16; x += T) {
            const int r = x / 16, cc = x % 16;
            if (tm[(j + 1 + r / 16) * nt + j]) st_c(&S[(size_t)(16 * (j + 1) + r) * N + 16 * j + cc], PT[cc * m + r]);
        }
        if (t < 16) {
            st_c(&Dg[16 * j + t], DP[t]);
            st_c(&Yg[16 * j + t], YP[t]);
        }
#if MAM_MW_DEFER
        pending = j;
#else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) st_ci(&mw[8 + j], tag);
#endif
        mprev = m;
        if (++jp == nt) break;
    }
    if (pending >= 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) st_ci(&mw[8 + pending], tag);
    }
    if (t == 0 && G == 1) st_ci(&mw[1], base + nt);   // (no helper made the last claim)
    // the backward substitution (every panel is this workgroup's own)
    LM& lm = *d.lm;
    __syncthreads();
    const int fl = ld_ci(&mw[2]);
    if (t == 0) lm.fail = fl != 0;
    if (fl) return true;
    inv_l1();
    double* Z = PT;
    for (int i = t; i < N; i += T) Z[i] = ld_pub(&Yg[i]) / ld_pub(&Dg[i]);
    __syncthreads();
    for (int k = nt - 1; k >= 0; k--) {
        dbl4 Q[RT];
#pragma unroll
        for (int u = 0; u < RT; u++) {
            const int i = wid + NW * u;
            Q[u] = dbl4{0.0, 0.0, 0.0, 0.0};
            if (i < k && tm[k * nt + i]) {
#pragma unroll
                for (int r = 0; r < 4; r++) Q[u][r] = ld_pub(&S[(size_t)(16 * k + rq + 4 * r) * N + 16 * i + col]);
            }
        }
        if (wid == 0) {
            double cl[NB];
#pragma unroll
            for (int jj = 0; jj < NB; jj++)
                cl[jj] = (lane < NB && jj > lane) ? ld_pub(&S[(size_t)(16 * k + jj) * N + 16 * k + lane]) : 0.0;
            double v = lane < NB ? Z[16 * k + lane] : 0.0;
#pragma unroll
            for (int jj = NB - 1; jj >= 0; jj--) {
                const double xj = bcast16_d(v, jj);
                if (lane < jj) v = fma(-cl[jj], xj, v);
            }
            if (lane < NB) Z[16 * k + lane] = v;
        }
        __syncthreads();
        const double y0 = Z[16 * k + rq], y1 = Z[16 * k + rq + 4], y2 = Z[16 * k + rq + 8], y3 = Z[16 * k + rq + 12];
#pragma unroll
        for (int u = 0; u < RT; u++) {
            const int i = wid + NW * u;
            if (i >= k || !tm[k * nt + i]) continue;
            double p = Q[u][0] * y0;
            p = fma(Q[u][1], y1, p);
            p = fma(Q[u][2], y2, p);
            p = fma(Q[u][3], y3, p);
            p += __shfl_xor(p, 16, 64);
            p += __shfl_xor(p, 32, 64);
            if (rq == 0) Z[16 * i + col] -= p;
        }
        __syncthreads();
    }
    for (int i = t; i < n; i += T) d.x[6 * (size_t)d.iperm[i / 6] + i % 6] = Z[i];   // (pose order)
    return true;
}

#ifndef MAM_MW_LOOKAHEAD
#define MAM_MW_LOOKAHEAD 1   // (ring batch of 32: 13.4 -> 12.8 ms against the chain form, same box)
#endif
__device__ __forceinline__ bool mw_takes(const Prob& d, const LMHead& hd) {
    return d.Np > 0 && !hd.tiles_lds && d.nt <= MW_NT_MAX;
}
// grid (G x Q rounded up to 8) x MW_T: the column-chain form's workgroups, a problem's G on one XCD (block b on
// XCD b mod 8), for the dense problems it takes (k_ldlt_any, launched before with mw_on, leaves them alone)
__global__ __launch_bounds__(MW_T) void k_ldlt_mw(const Prob* __restrict__ probs, int Q, int G) {
    extern __shared__ __attribute__((aligned(16))) double lds_dyn[];
    __shared__ LdltShared sh;
    const int xcd = blockIdx.x % 8, idx = blockIdx.x / 8, p = (idx / G) * 8 + xcd;
    if (p >= Q) return;
    const Prob& d = probs[p];
    const LMHead hd = lm_head(d.lm);
    if (hd.status || hd.done || !mw_takes(d, hd)) return;
#if MAM_MW_LOOKAHEAD
    if (ldlt_mw_la<MW_T>(d, lds_dyn, sh, G)) {
#else
    if (ldlt_mw<MW_T>(d, lds_dyn, sh, G)) {
#endif
        __syncthreads();
        pose_epilogue<MW_T>(d, *d.lm, hd.cur, d.x, trial_lambda(hd));
    }
}

template <bool use_lds>
__global__ __launch_bounds__(LDLT_THREADS) void k_ldlt_any(const Prob* __restrict__ probs, int reg_nt_max, int mw_on) {
    extern __shared__ __attribute__((aligned(16))) double lds_dyn[];
    __shared__ LdltShared sh;
    const Prob& d = probs[blockIdx.x];
    const LMHead hd = lm_head(d.lm);
    if (hd.status || hd.done) return;
    if (d.Np > 0 && !hd.tiles_lds && d.nt <= reg_nt_max) return;   // k_ldlt_reg's
    if (mw_on && mw_takes(d, hd)) return;                          // k_ldlt_mw's
    LM& lm = *d.lm;
    if (d.Np == 0) {
        if (threadIdx.x == 0) lm.fail = 0;
    } else if (hd.tiles_lds) {
        ldlt_tiles(d, lds_dyn, sh, hd);
    } else {
        ldlt_global<use_lds>(d, lds_dyn, sh);
    }
    __syncthreads();
    pose_epilogue<LDLT_THREADS>(d, lm, hd.cur, d.x, trial_lambda(hd));
}

// grid (Q) x 256: end of a trial — levenberg.cpp:108-158 (rho, accept / reject, lambda), then the iteration-end
// tests of levenberg.cpp:159-168 and sparse_optimizer.cpp:381-409. (Run instead by the last workgroup of the trial's
// k_linearize, the kernel boundary replaced by a release / acquire per workgroup, the batch of 32 took 5.6 -> 9.5 ms:
// every workgroup's agent-scope release writes its L2 back.)
// grid (Q) x 256: end of a trial — ctl_step on the trial's chi2 and computeScale. (Run instead by the last workgroup of
// the trial's k_linearize, the kernel boundary replaced by a release / acquire per workgroup, the batch of 32 took
// 5.6 -> 9.5 ms: every workgroup's agent-scope release writes its L2 back. Folded into the next trial's k_point_sys
// for a single window — every workgroup computing it from the same partials, the last one writing the state back —
// the lone window took 1.278 -> 1.318 ms: k_point_sys grew 7.6 us, more than the launch it saved.)
__global__ __launch_bounds__(RED) void k_ctl_end(const Prob* __restrict__ probs) {
    constexpr int T = RED;
    __shared__ double s[RED];
    const Prob& d = probs[blockIdx.x];
    const LMHead hd = lm_head(d.lm);
    if (hd.status || hd.done) return;
    double tempChi, scale0;
    trial_sums<T>(d, s, &tempChi, &scale0);
    if (threadIdx.x != 0) return;
    ctl_step(*d.lm, hd, tempChi, scale0);
}

// grid (ceil(E/256), Q): isDepthPositive of the final estimate
__global__ __launch_bounds__(256) void k_depth(const Prob* __restrict__ probs) {
    const Prob& d = probs[blockIdx.y];
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= d.E || d.lm->status) return;
    const int c = d.lm->cur;
    double Xc[3];
    map_point(d.pose[c] + 7 * (size_t)d.edge_pose[e], d.pt[c] + 3 * (size_t)d.edge_point[e], Xc);
    d.depth[e] = Xc[2] > 0.0;
}

}  // namespace lba
}  // namespace mam

// ==================================================================================================== host
using mam::DevBuf;
using mam::lba::LM;
using mam::lba::Prob;

struct mam_lba_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    size_t ldlt_lds_budget = 0;   // dynamic LDS the factorization may use (panel staging)
    mam::PinnedBuf staging;       // host mirror of the uploaded inputs (host API: one copy per solve)
    mam::PinnedBuf lm_host;       // LM states read back once per chunk of slots
    mam::StageTimer timer{4};
    DevBuf<uint8_t> arena;        // per-problem structure, state and scratch of the current batch
    DevBuf<uint8_t> io;           // host API: inputs + outputs of the one problem
    hipStream_t up_stream = nullptr;   // host API: the observations' upload beside the structure build
    hipEvent_t up_done = nullptr;
    DevBuf<uint8_t> hdr;          // Prob[Q] | LM[Q] | Outs[Q] of the current batch
    DevBuf<int2> blk_pairs;       // the S blocks' landmark pairs of the current batch
    static constexpr int kMaxGroups = 4;
    hipStream_t gstream[kMaxGroups - 1] = {};   // groups 1.. of a split batch (created on first use, caller's priority)
    hipEvent_t ev_start = nullptr, ev_done[kMaxGroups - 1] = {};
    std::vector<uint32_t> cu_mask;   // the group streams' CU mask (mam_lba_set_cu_mask; empty: every CU)
    double trials_ema = 8.0;      // slots enqueued before the first read-back (tracks the trials solves take)
};

namespace {

constexpr size_t kAlign = 256;
size_t al(size_t b) { return (b + kAlign - 1) & ~(kAlign - 1); }

struct Carver {
    uint8_t* base;
    size_t off = 0;
    template <typename T>
    T* take(size_t n) {
        T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;   // (base null: a dry run counting bytes)
        off += al(n * sizeof(T));
        return p;
    }
};

void carve_scratch(Carver& cv, Prob& d) {
    const size_t nx = 6 * (size_t)d.Np + 3 * (size_t)d.L;
    d.pose_h = cv.take<int32_t>(d.P);
    d.hpose = cv.take<int32_t>(d.Np);
    d.pe_off = cv.take<int32_t>(d.L + 1);
    d.pe_idx = cv.take<int32_t>(d.E);
    d.slot_hp = cv.take<int32_t>(d.E);
    d.emeta = cv.take<int4>(d.E);
    d.qe_off = cv.take<int32_t>(d.Np + 1);
    d.qe_idx = cv.take<int32_t>(d.E);
    d.cnt = cv.take<int32_t>(d.L + d.Np);
    d.eidx = cv.take<int32_t>((size_t)d.Np * d.L);
    d.pairmask = cv.take<uint8_t>((size_t)d.Np * d.Np);
    d.pm_rows = cv.take<unsigned long long>(64);
    d.blk_off = cv.take<int32_t>((size_t)d.Np * d.Np + 1);
    d.nt = d.npad / mam::lba::NB;
    d.tmask = cv.take<uint8_t>((size_t)d.nt * d.nt);
    d.tslot = cv.take<int16_t>((size_t)d.nt * d.nt);
    d.tlist = cv.take<int16_t>((size_t)d.nt * (d.nt + 1));
    d.clist_g = cv.take<int8_t>((size_t)std::max(d.nt, 1) * 40);
    d.rlist_g = cv.take<int8_t>((size_t)std::max(d.nt, 1) * 40);
    d.ccnt_g = cv.take<uint8_t>(2 * (size_t)std::max(d.nt, 1));
    d.perm = cv.take<int16_t>((size_t)std::max(d.Np, 1));
    d.iperm = cv.take<int16_t>((size_t)std::max(d.Np, 1));
    d.order_g = cv.take<int8_t>(40);
    d.pool = cv.take<double>((size_t)d.nt * (d.nt + 1) / 2 * 256);
    d.pose[0] = cv.take<double>(7 * (size_t)d.P);
    d.pose[1] = cv.take<double>(7 * (size_t)d.P);
    d.pt[0] = cv.take<double>(3 * (size_t)d.L);
    d.pt[1] = cv.take<double>(3 * (size_t)d.L);
    d.err = cv.take<double>(2 * (size_t)d.E);
    d.jac = cv.take<double>(21 * (size_t)d.E);
    const int pwm = 2;   // (the fewest points per workgroup any launch takes)
    const size_t np = (size_t)std::max((d.E + 63) / 64, (d.L + pwm - 1) / pwm) + 1;
    d.part = cv.take<double>(np);
    d.part0 = cv.take<double>(np);
    d.part_s = cv.take<double>(np);
    d.hpl = cv.take<double>(18 * (size_t)d.E);
    d.bdinv = cv.take<double>(18 * (size_t)d.E);
    d.coef = cv.take<double>(6 * (size_t)d.E);
    d.Hpp = cv.take<double>(36 * (size_t)mam::lba::POSE_SPLIT * d.Np);
    d.bp = cv.take<double>(6 * (size_t)mam::lba::POSE_SPLIT * d.Np);
    d.Hll = cv.take<double>(9 * (size_t)d.L);
    d.b = cv.take<double>(nx);
    d.Dinv = cv.take<double>(9 * (size_t)d.L);
    d.S = cv.take<double>((size_t)d.npad * d.npad);
    d.x = cv.take<double>(nx);
    d.bs = cv.take<double>(d.npad);
    d.ws = cv.take<double>(mam::lba::ldlt_ws_doubles(d.npad));
    d.mw = cv.take<int32_t>(mam::lba::MW_INTS);
    d.depth = cv.take<uint8_t>(d.E);
}

// Arena bytes of one problem's structure, state and scratch (the inputs and outputs live elsewhere): a dry run of
// carve_scratch, so the size and the carve cannot drift apart (a hand-kept formula once missed the pose sums'
// POSE_SPLIT partials and a batch's problems overran into their neighbours' structure)
size_t scratch_bytes(const Prob& d0) {
    Prob d = d0;
    Carver cv{nullptr};
    carve_scratch(cv, d);
    return cv.off;
}

// Output pointers of a batch problem (device memory); chi2 / depth may be NULL
struct Outs {
    double* q;
    double* t;
    double* xyz;
    double* chi2;
    uint8_t* depth;
};

}  // namespace

namespace mam {
namespace lba {

// grid (ceil(max(E, P, L)/256), Q): results of the final estimate (cur): poses split into q / t, points, per-edge
// chi2() = e^T Omega e of the last computed errors (level-0 edges only) and isDepthPositive()
__global__ __launch_bounds__(256) void k_finish(const Prob* __restrict__ probs, const Outs* __restrict__ outs) {
    const Prob& d = probs[blockIdx.y];
    const Outs& o = outs[blockIdx.y];
    if (d.lm->status) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int c = d.lm->cur;
    if (i < d.P) {
        const double* T = d.pose[c] + 7 * (size_t)i;
        for (int k = 0; k < 4; k++) o.q[4 * (size_t)i + k] = T[k];
        for (int k = 0; k < 3; k++) o.t[3 * (size_t)i + k] = T[4 + k];
    }
    if (i < d.L)
        for (int k = 0; k < 3; k++) o.xyz[3 * (size_t)i + k] = d.pt[c][3 * (size_t)i + k];
    if (i < d.E) {
        if (o.chi2 && !(d.active && !d.active[i])) {
            const double w = d.edge_w[i], e0 = d.err[2 * i], e1 = d.err[2 * i + 1];
            o.chi2[i] = e0 * (w * e0) + e1 * (w * e1);
        }
        if (o.depth) {
            double Xc[3];
            map_point(d.pose[c] + 7 * (size_t)d.edge_pose[i], d.pt[c] + 3 * (size_t)d.edge_point[i], Xc);
            o.depth[i] = Xc[2] > 0.0;
        }
    }
}

}  // namespace lba
}  // namespace mam

namespace {

// The shared driver: Q problems whose inputs (id-ordered) are already in device memory, described by hp[q] (input
// pointers, dimensions, delta, iterations in lm0[q]). Builds the structure on the device, runs the LM slots, writes
// the outputs and fills the host-side scalars of res[q] (iterations, trials, chi2s, status).
// before_lin (may be empty): called once the structure build is enqueued, before the first linearisation; it may
// enqueue work the linearisation needs (mam_lba_solve: the observations' upload, overlapped with the build) and
// returns an event the stream then waits on (nullptr: none) or sets rc.
int run_batch(mam_lba_ctx* c, std::vector<Prob>& hp, std::vector<LM>& lm0, const std::vector<Outs>& outs,
              const volatile uint8_t* stop_flag, hipStream_t s, mam_lba_result* res,
              const std::function<hipEvent_t(int*)>& before_lin = {}) {
    using namespace mam::lba;
    const int Q = (int)hp.size();
    if (Q == 0) return MAM_OK;
    size_t bytes = 0;
    int maxE = 0, maxL = 0, maxP = 0, maxNp = 0, maxLb = 0;
    size_t max_lds = 0;
    bool lds_ok = true;
    for (auto& d : hp) {
        d.npad = ldlt_pad(6 * d.Np);
        bytes += scratch_bytes(d);
        maxE = std::max(maxE, d.E);
        maxL = std::max(maxL, d.L);
        maxP = std::max(maxP, d.P);
        maxNp = std::max(maxNp, d.Np);
        maxLb = std::max(maxLb, (d.L + 255) / 256 + d.Np);
        max_lds = std::max(max_lds, ldlt_lds_bytes(d.npad));
    }
    if (max_lds > c->ldlt_lds_budget) lds_ok = false;
    if (ldlt_pad(6 * maxNp) / NB > LDLT_TM_MAX) lds_ok = false;   // the LDS path keeps the tile mask in LDS too
    // size bounds before any allocation: the dense pose x landmark edge table (Np L int32) and S (npad^2 f64) of one
    // problem stay under 4 GiB each, and the batch's scratch fits the device's free memory
    for (auto& d : hp) {
        const double eidx_b = 4.0 * d.Np * (double)d.L, s_b = 8.0 * d.npad * (double)d.npad;
        if (eidx_b > 4294967296.0 || s_b > 4294967296.0) {
            mam::set_last_error("LBA problem too large for the dense solve: " + std::to_string(d.Np) +
                                " optimised poses x " + std::to_string(d.L) + " points (pose x landmark table " +
                                std::to_string((long long)(eidx_b / 1048576)) + " MiB, S " +
                                std::to_string((long long)(s_b / 1048576)) + " MiB; bound 4096 MiB each)");
            return MAM_ERR_CAPACITY;
        }
    }
    if (bytes + kAlign > c->arena.n) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && bytes + kAlign > free_b + c->arena.n) {
            mam::set_last_error("LBA batch scratch of " + std::to_string(bytes >> 20) + " MiB exceeds the device's free " +
                                std::to_string(free_b >> 20) + " MiB");
            return MAM_ERR_CAPACITY;
        }
    }
    // the S blocks' landmark pairs: at most (edges of the optimised poses) x (optimised poses observing the landmark)
    // per block column, so E Np per problem bounds them. Below kPairBoundBytes the buffer is sized by that bound up
    // front (no read-back of the counts before the fill); above it (map-scale graphs, where E Np overestimates the
    // sum over landmarks of their observers squared by orders of magnitude) the exact counts are read back after
    // k_blk_scan and the buffer sized by them
    // (2 GiB of 288: a batch of 32 dense c2 windows bounds at ~490 MB and takes the up-front form; at 256 MB it took
    // the read-back form: 2 Q 4-byte copies and two host synchronisations a solve on LocalMapping's stream)
    constexpr size_t kPairBoundBytes = (size_t)2 << 30;
    std::vector<size_t> pair_cap(Q);
    size_t npairs = 0;
    for (int q = 0; q < Q; q++) {
        pair_cap[q] = (size_t)hp[q].E * (size_t)std::max(hp[q].Np, 1);
        npairs += pair_cap[q];
    }
    const bool exact_pairs = npairs * sizeof(int2) > kPairBoundBytes;
    if (int rc = c->arena.alloc(bytes + kAlign)) return rc;
    if (!exact_pairs)
        if (int rc = c->blk_pairs.alloc(std::max<size_t>(npairs, 1))) return rc;
    // one device block and one pinned block of the same layout: Prob[Q] | LM[Q] | Outs[Q], one upload
    const size_t pb = al(sizeof(Prob) * Q), lb = al(sizeof(LM) * Q), ob = al(sizeof(Outs) * Q);
    if (int rc = c->hdr.alloc(pb + lb + ob)) return rc;
    if (int rc = c->lm_host.alloc(pb + lb + ob)) return rc;
    Prob* const P = reinterpret_cast<Prob*>(c->hdr.p);
    LM* const lms_d = reinterpret_cast<LM*>(c->hdr.p + pb);
    Outs* const outs_d = reinterpret_cast<Outs*>(c->hdr.p + pb + lb);
    Carver cv{c->arena.p};
    for (auto& d : hp) carve_scratch(cv, d);
    size_t base = 0;
    // points per k_point_sys / k_point_trial workgroup: PW_SMALL for a lone window whose points have many observations
    // (a covisibility ring window, ~12 a point: 1.23 -> 1.11 ms), PW otherwise (a window of ~8 observations a point
    // fills PW = 8 points' 64 slots exactly: 1.23 ms, 1.28 at PW_SMALL; batches are throughput-bound: PW)
    size_t sumE = 0, sumL = 0;
    for (int q = 0; q < Q; q++) {
        sumE += (size_t)hp[q].E;
        sumL += (size_t)hp[q].L;
    }
    int pw_batch = (Q <= 2 && sumL > 0 && (double)sumE > 10.0 * (double)sumL) ? PW_SMALL : PW;
    if (const char* e = std::getenv("MAM_LBA_PW")) {   // experiments: force 2, 4 or 8 points per workgroup
        const int v = std::atoi(e);
        if (v == 2 || v == 4 || v == 8) pw_batch = v;
    }
    for (int q = 0; q < Q; q++) {
        hp[q].lm = lms_d + q;
        hp[q].blk_pair = exact_pairs ? nullptr : c->blk_pairs.p + base;
        hp[q].pair_fixed = exact_pairs ? 0 : 1;
        hp[q].pw = pw_batch;   // (the launches below take the same)
        base += pair_cap[q];
    }
    std::memcpy(c->lm_host.p, hp.data(), sizeof(Prob) * Q);
    std::memcpy(c->lm_host.p + pb, lm0.data(), sizeof(LM) * Q);
    std::memcpy(c->lm_host.p + pb + lb, outs.data(), sizeof(Outs) * Q);
    MAM_HIP(hipMemcpyAsync(c->hdr.p, c->lm_host.p, pb + lb + ob, hipMemcpyHostToDevice, s));
    // the factorization's dynamic LDS: the tile pool budget (k_struct_tiles keeps a problem's pool + y within it) and
    // the HBM form's panel workspace, the larger
    size_t ldlt_dyn = c->ldlt_lds_budget;
    if (lds_ok) ldlt_dyn = std::max(ldlt_dyn, max_lds);
    // the register form (k_ldlt_reg) for the problems whose nt it holds in registers + the LDS budget, unless they
    // fit the LDS tile pool (decided on the device), with MAM_LBA_REG=1; otherwise every problem goes to k_ldlt_any
    // (while the tiles neither registers nor the LDS left over hold — read-modify-written in S — number at most
    // MAM_LBA_REG_GLOBAL, default 64)
    int reg_nt_max = 0, reg_nt_used = 0;
    auto reg_over_lds = [](int nt) {   // tiles past the registers, and the LDS they take (+ the 16-B alignment)
        const int over = std::max(0, nt * (nt + 1) / 2 - (REG_T / 64) * REG_RT);
        return std::make_pair(over, (size_t)over * 256 * sizeof(double) + 16);
    };
    {
        const char* rv = std::getenv("MAM_LBA_REG");
        const char* gv = std::getenv("MAM_LBA_REG_GLOBAL");
        const int gmax = gv ? std::atoi(gv) : 64;
        if (rv && rv[0] == '1')   // (off by default until it beats the HBM form: DESIGN §6)
            while (reg_nt_max < LDLT_TM_MAX) {
                const int nt = reg_nt_max + 1;
                const size_t base = ldlt_reg_lds_bytes(nt);
                if (base + 16 > c->ldlt_lds_budget) break;
                const auto ov = reg_over_lds(nt);
                const int fit = (int)((c->ldlt_lds_budget - base - 16) / (256 * sizeof(double)));
                if (ov.first - fit > gmax) break;
                reg_nt_max = nt;
            }
        for (auto& d : hp)
            if (d.Np > 0 && d.npad / NB <= reg_nt_max) reg_nt_used = std::max(reg_nt_used, d.npad / NB);
        if (reg_nt_used == 0) reg_nt_max = 0;
    }
    const size_t reg_dyn = reg_nt_used ? std::min(c->ldlt_lds_budget, ldlt_reg_lds_bytes(reg_nt_used) +
                                                                          reg_over_lds(reg_nt_used).second)
                                       : 0;
    // the column-chain form (ldlt_mw) for the problems whose every tile would not fit the LDS tile pool (the device
    // decides per problem: a sparse pattern still goes to the pool); MAM_LBA_MW=0 leaves them to the HBM form
    // (batches only: a lone window's chain of column handoffs is slower than one workgroup's HBM form, 2.94 against
    // 2.77 ms for a c2 ring window; MAM_LBA_MW=2 takes lone problems too)
    bool mw_on = false;
    size_t mw_dyn = 0;
    {
        const char* mv = std::getenv("MAM_LBA_MW");
        int cand = 0;
        if (!(mv && mv[0] == '0') && reg_nt_max == 0)
            for (auto& d : hp) {
                const int nt = d.npad / NB;
                if (d.Np > 0 && nt <= MW_NT_MAX &&
                    (size_t)nt * (nt + 1) / 2 * 256 * sizeof(double) + (size_t)d.npad * sizeof(double) > c->ldlt_lds_budget) {
                    cand++;
                    mw_dyn = std::max(mw_dyn, ldlt_mw_lds_bytes(d.npad));
                }
            }
        mw_on = cand >= ((mv && mv[0] == '2') ? 1 : 2);
    }
    const dim3 gE((maxE + 255) / 256 > 0 ? (maxE + 255) / 256 : 1, Q);
    const dim3 gE64((maxE + EW - 1) / EW > 0 ? (maxE + EW - 1) / EW : 1, Q);
    {
        mam::StageTimer::Scope sc(&c->timer, s, 0);
        hipLaunchKernelGGL(k_struct_init, dim3(8, Q), dim3(SB), 0, s, P);
        hipLaunchKernelGGL(k_struct_count, gE, dim3(256), 0, s, P);
        hipLaunchKernelGGL(k_struct_scan, dim3(1, Q), dim3(SB), 0, s, P);
        hipLaunchKernelGGL(k_struct_scatter, gE, dim3(256), 0, s, P);
        hipLaunchKernelGGL(k_struct_sort, dim3(std::max(maxLb, 1), Q), dim3(256), 0, s, P);
        hipLaunchKernelGGL(k_struct_tiles, dim3(Q), dim3(SB), 0, s, P, (int)c->ldlt_lds_budget);
        // the S blocks' landmark pairs: counts, offsets, the pairs
        const dim3 gB(std::max(maxNp * maxNp, 1), Q);
        if (exact_pairs) {   // (else the blocks sit at fixed offsets of the E Np buffer: k_blk_fill counts them)
            hipLaunchKernelGGL(k_blk_count, gB, dim3(64), 0, s, P);
            hipLaunchKernelGGL(k_blk_scan, dim3(1, Q), dim3(SB), 0, s, P);
        }
        if (exact_pairs) {
            // the totals at blk_off[Np * Np] (a problem whose structure failed keeps status != 0 and fills nothing)
            std::vector<int32_t> tot(Q, 0);
            for (int q = 0; q < Q; q++)
                MAM_HIP(hipMemcpyAsync(&tot[q], hp[q].blk_off + (size_t)hp[q].Np * hp[q].Np, sizeof(int32_t),
                                       hipMemcpyDeviceToHost, s));
            MAM_HIP(hipStreamSynchronize(s));
            size_t n_exact = 0;
            std::vector<size_t> off(Q);
            for (int q = 0; q < Q; q++) {
                off[q] = n_exact;
                n_exact += (size_t)std::min<size_t>((size_t)std::max(tot[q], 0), pair_cap[q]);
            }
            if (int rc = c->blk_pairs.alloc(std::max<size_t>(n_exact, 1))) return rc;
            std::vector<int2*> ptr(Q);
            for (int q = 0; q < Q; q++) {
                ptr[q] = c->blk_pairs.p + off[q];
                MAM_HIP(hipMemcpyAsync(&P[q].blk_pair, &ptr[q], sizeof(int2*), hipMemcpyHostToDevice, s));
            }
            MAM_HIP(hipStreamSynchronize(s));
        }
        hipLaunchKernelGGL(k_blk_fill, gB, dim3(64), 0, s, P);
        // iteration 0's linearisation and system at the initial state (lambda_0 needs its max |diag(H)|), the initial
        // chi2; the first trial's k_point_sys then starts from this system
        const dim3 gSys((maxL + 63) / 64 + maxNp * POSE_SPLIT > 0 ? (maxL + 63) / 64 + maxNp * POSE_SPLIT : 1, Q);
        if (before_lin) {
            int rc = MAM_OK;
            const hipEvent_t ev = before_lin(&rc);
            if (rc) return rc;
            if (ev) MAM_HIP(hipStreamWaitEvent(s, ev, 0));
        }
        hipLaunchKernelGGL(k_linearize, gE64, dim3(EW), 0, s, P);
        hipLaunchKernelGGL(k_sys, gSys, dim3(64), 0, s, P);
        hipLaunchKernelGGL(k_ctl_init, dim3(Q), dim3(RED), 0, s, P);
    }
    const int pw = pw_batch;
    const int nbp = std::max((maxL + pw - 1) / pw, 1);
    const dim3 gPts(nbp + maxNp * POSE_SPLIT, Q), gTri(nbp, Q);
    const dim3 gBlk(maxNp * (maxNp + 1) / 2 + maxNp > 0 ? maxNp * (maxNp + 1) / 2 + maxNp : 1, Q);
    const int maxPL = std::max(maxP, maxL);
    // The batch runs as G interleaved groups on G streams: one group's latency-bound factorization (one workgroup
    // per problem) overlaps the other groups' throughput kernels. Every kernel indexes its problems from the Prob
    // pointer it is given, so a group is the sub-array P + first with Q_g problems. MAM_LBA_SPLIT=<G> overrides
    // (1 disables).
    const char* sp = std::getenv("MAM_LBA_SPLIT");
    int G = Q < 4 ? 1 : 2;   // batch of 32 world windows: 8.56 / 7.92 / 7.76 / 9.10 ms at G = 1 / 2 / 3 / 4; c2: 2
    if (sp && sp[0] >= '1' && sp[0] <= '9') G = std::max(1, std::min({mam_lba_ctx::kMaxGroups, Q, sp[0] - '0'}));
    hipStream_t sg[mam_lba_ctx::kMaxGroups] = {s, s, s, s};
    if (G > 1) {
        int prio = 0;
        if (hipStreamGetPriority(s, &prio) != hipSuccess) prio = 0;
        if (!c->ev_start) MAM_HIP(hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming));
        for (int g = 1; g < G; g++) {
            if (!c->gstream[g - 1] && !c->cu_mask.empty()) {
                MAM_HIP(hipExtStreamCreateWithCUMask(&c->gstream[g - 1], (uint32_t)c->cu_mask.size(), c->cu_mask.data()));
                MAM_HIP(hipEventCreateWithFlags(&c->ev_done[g - 1], hipEventDisableTiming));
            } else if (!c->gstream[g - 1]) {
                if (hipStreamCreateWithPriority(&c->gstream[g - 1], hipStreamNonBlocking, prio) != hipSuccess) {
                    (void)hipGetLastError();
                    MAM_HIP(hipStreamCreateWithFlags(&c->gstream[g - 1], hipStreamNonBlocking));
                }
                MAM_HIP(hipEventCreateWithFlags(&c->ev_done[g - 1], hipEventDisableTiming));
            }
            sg[g] = c->gstream[g - 1];
        }
        MAM_HIP(hipEventRecord(c->ev_start, s));   // the structure build precedes every group
        for (int g = 1; g < G; g++) MAM_HIP(hipStreamWaitEvent(sg[g], c->ev_start, 0));
    }
    auto slot_g = [&](int g) {
        const int q0 = g * Q / G, q1 = (g + 1) * Q / G, Qg = q1 - q0;
        const Prob* Pg = P + q0;
        hipStream_t st = sg[g];
        const dim3 gPtsg(gPts.x, Qg), gTrig(gTri.x, Qg), gBlkg(gBlk.x, Qg);
        // the column-chain form's workgroups when a problem may be dense past the LDS tile pool (decided on the device)
        // (a lone problem: a workgroup per column, every column's chain at once)
        int mwg = MW_G;
        if (Qg == 1) mwg = std::max(MW_G, std::min(hp[q0].npad / NB, MW_NT_MAX));
        const int mwb = mw_on ? mwg * ((Qg + 7) / 8 * 8) : 0;
        mam::StageTimer* tm = g == 0 ? &c->timer : nullptr;   // stage times: the first half's kernels
        {
            mam::StageTimer::Scope sc(tm, st, 0);
            if (pw == 2)
                hipLaunchKernelGGL(k_point_sys<2>, gPtsg, dim3(64), 0, st, Pg);
            else if (pw == 4)
                hipLaunchKernelGGL(k_point_sys<4>, gPtsg, dim3(64), 0, st, Pg);
            else
                hipLaunchKernelGGL(k_point_sys<8>, gPtsg, dim3(64), 0, st, Pg);
        }
        {
            mam::StageTimer::Scope sc(tm, st, 1);
            if (Qg >= 4)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_schur_blk<MAM_SCHUR_T_BATCH, false>), gBlkg, dim3(MAM_SCHUR_T_BATCH), 0,
                                   st, Pg);
            else
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_schur_blk<MAM_SCHUR_T, (bool)MAM_SCHUR_FULL>), gBlkg, dim3(MAM_SCHUR_T), 0,
                                   st, Pg);
        }
        {
            mam::StageTimer::Scope sc(tm, st, 2);
            if (lds_ok)
                hipLaunchKernelGGL(k_ldlt_any<true>, dim3(Qg), dim3(LDLT_THREADS), ldlt_dyn, st, Pg, reg_nt_max,
                                   (int)mw_on);
            else
                hipLaunchKernelGGL(k_ldlt_any<false>, dim3(Qg), dim3(LDLT_THREADS), ldlt_dyn, st, Pg, reg_nt_max,
                                   (int)mw_on);
            if (mw_on) hipLaunchKernelGGL(k_ldlt_mw, dim3(mwb), dim3(MW_T), mw_dyn, st, Pg, Qg, mwg);
            if (reg_nt_max)
                hipLaunchKernelGGL(k_ldlt_reg, dim3(Qg), dim3(REG_T), reg_dyn, st, Pg, reg_nt_max,
                                   reg_dyn);
        }
        {
            mam::StageTimer::Scope sc(tm, st, 3);
            if (pw == 2)
                hipLaunchKernelGGL(k_point_trial<2>, gTrig, dim3(64), 0, st, Pg);
            else if (pw == 4)
                hipLaunchKernelGGL(k_point_trial<4>, gTrig, dim3(64), 0, st, Pg);
            else
                hipLaunchKernelGGL(k_point_trial<8>, gTrig, dim3(64), 0, st, Pg);
            hipLaunchKernelGGL(k_ctl_end, dim3(Qg), dim3(RED), 0, st, Pg);
        }
    };
    auto slot = [&]() {
        for (int g = 0; g < G; g++) slot_g(g);
    };
    auto join = [&]() -> int {   // the other groups' work before anything the first stream does next
        for (int g = 1; g < G; g++) {
            MAM_HIP(hipEventRecord(c->ev_done[g - 1], sg[g]));
            MAM_HIP(hipStreamWaitEvent(s, c->ev_done[g - 1], 0));
        }
        return MAM_OK;
    };
    auto stopped = [&]() { return stop_flag && *stop_flag; };
    // Every slot is one Levenberg trial of every unfinished problem, so a solve needs at most iterations x 10 slots;
    // the host reads the states back once per chunk (the first chunk sized by the trials recent solves took). Each
    // chunk ends with k_finish (the outputs of the current state: rewritten by the next chunk's if there is one), so
    // a solve that ends within its first chunk costs one host round trip.
    int max_slots = 0;
    for (auto& l : lm0) max_slots = std::max(max_slots, 10 * std::max(l.iterations, 0));
    int chunk = std::max(1, (int)std::lround(c->trials_ema));   // nearest: a ceil of 9.02 enqueued a 10th slot
    int enq = 0;
    LM* lh = reinterpret_cast<LM*>(c->lm_host.p + pb);
    bool was_stopped = false;
    const dim3 gFin(std::max({(maxE + 255) / 256, (maxPL + 255) / 256, 1}), Q);
    auto finish_and_read = [&]() -> int {
        if (int rc = join()) return rc;
        hipLaunchKernelGGL(mam::lba::k_finish, gFin, dim3(256), 0, s, P, outs_d);
        MAM_HIP(hipGetLastError());
        MAM_HIP(hipMemcpyAsync(lh, lms_d, sizeof(LM) * Q, hipMemcpyDeviceToHost, s));
        MAM_HIP(hipStreamSynchronize(s));
        return MAM_OK;
    };
    bool read = false;   // lh (and the outputs) hold the state after the last enqueued slot
    while (enq < max_slots) {
        if (stopped()) { was_stopped = true; break; }
        const int k = std::min(chunk, max_slots - enq);
        for (int i = 0; i < k; i++) slot();
        enq += k;
        MAM_HIP(hipGetLastError());
        if (int rc = finish_and_read()) return rc;
        read = true;
        bool all = true;
        for (int q = 0; q < Q; q++) all = all && (lh[q].done || lh[q].status);
        if (all) break;
        read = false;   // more slots follow
        chunk = 2;
    }
    if (!read)
        if (int rc = finish_and_read()) return rc;
    int max_trials = 0;
    for (int q = 0; q < Q; q++) {
        res[q].iterations = lh[q].its;
        res[q].lm_trials = lh[q].trials;
        res[q].initial_chi2 = lh[q].initialChi;
        res[q].final_chi2 = lh[q].acceptedChi;   // activeRobustChi2 of the final state
        res[q].status = lh[q].status ? lh[q].status : ((was_stopped || stopped()) ? 1 : 0);
        max_trials = std::max(max_trials, lh[q].trials);
    }
    if (!was_stopped) c->trials_ema = 0.75 * c->trials_ema + 0.25 * std::max(1, max_trials);
#ifdef MAM_LDLT_TRACE
    {
        long long tr[40][8];
        MAM_HIP(hipMemcpyFromSymbol(tr, HIP_SYMBOL(mam::lba::g_ltrace), sizeof(tr)));
        const int nt0 = hp[0].nt;
        const long long t0 = tr[0][2];
        for (int k = 0; k < nt0 && k < 40; k++)
            fprintf(stderr, "ltrace col %2d: dwait %7lld ddone %7lld count %7lld load %7lld panel %7lld flag %7lld back %7lld\n",
                    k, tr[k][6] - t0, tr[k][0] - t0, tr[k][1] - t0, tr[k][2] - t0, tr[k][3] - t0, tr[k][4] - t0,
                    tr[k][5] - t0);
    }
#endif
#ifdef MAM_LDLT_PROFILE
    {
        unsigned long long h[8];
        MAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(mam::lba::g_lprof), sizeof(h)));
        const double w = (double)std::max(1ull, h[7]);
        fprintf(stderr, "ldlt cycles per WG: init %.0f B %.0f C1 %.0f C2 %.0f solve %.0f diag(w0) %.0f pull %.0f; WGs %llu\n",
                h[0] / w, h[1] / w, h[2] / w, h[3] / w, h[4] / w, h[5] / w, h[6] / w, h[7]);
    }
#endif
#ifdef MAM_SORT_PROFILE
    {
        MAM_HIP(hipStreamSynchronize(s));
        unsigned long long h[4];
        MAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(mam::lba::g_sortprof), sizeof(h)));
        fprintf(stderr, "struct_sort cycles per workgroup: points %.0f (%llu) poses %.0f (%llu)\n",
                h[0] / (double)std::max(1ull, h[2]), h[2], h[1] / (double)std::max(1ull, h[3]), h[3]);
    }
#endif
#ifdef MAM_MW_PROFILE
    {
        MAM_HIP(hipStreamSynchronize(s));
        unsigned long long h[8];
        MAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(mam::lba::g_mwprof), sizeof(h)));
        fprintf(stderr, "mw cycles (sum over workgroups): wait %.3g steps %.3g panel %.3g publish %.3g backward %.3g; "
                        "columns %llu k steps %llu; per step: wait %.0f update %.0f; per column: panel %.0f publish %.0f\n",
                (double)h[0], (double)h[1], (double)h[2], (double)h[3], (double)h[4], h[6], h[7],
                h[0] / (double)std::max(1ull, h[7]), h[1] / (double)std::max(1ull, h[7]),
                h[2] / (double)std::max(1ull, h[6]), h[3] / (double)std::max(1ull, h[6]));
    }
#endif
#ifdef MAM_REG_PROFILE
    {
        MAM_HIP(hipStreamSynchronize(s));
        unsigned long long h[8];
        MAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(mam::lba::g_rprof), sizeof(h)));
        const double w = (double)std::max(1ull, h[7]);
        int hist[64] = {0};
        for (auto& d : hp)
            if (d.Np > 0) hist[std::min(63, d.npad / NB)]++;
        for (int i = 0; i < 64; i++)
            if (hist[i]) fprintf(stderr, "nt %d: %d problems\n", i, hist[i]);
        fprintf(stderr, "reg ldlt cycles per WG: init %.0f stage %.0f diag %.0f panel %.0f update %.0f backward %.0f; "
                        "WGs %llu reg_nt_max %d\n", h[0] / w, h[1] / w, h[2] / w, h[3] / w, h[4] / w, h[5] / w, h[7],
                reg_nt_max);
    }
#endif
    return MAM_OK;
}

bool problem_ok(const mam_lba_problem* p) {
    if (!p || p->n_poses < 0 || p->n_points < 0 || p->n_edges < 0 || !p->cams || p->n_cams < 1) return false;
    if (p->cam_model != MAM_CAM_PINHOLE && p->cam_model != MAM_CAM_KANNALA_BRANDT8) return false;
    if ((p->n_poses > 0 && (!p->pose_fixed || !p->pose_q || !p->pose_t)) || (p->n_points > 0 && !p->point_xyz) ||
        (p->n_edges > 0 && (!p->edge_point || !p->edge_pose || !p->edge_obs || !p->edge_inv_sigma2)))
        return false;
    return true;
}

Prob desc_of(const mam_lba_problem* p) {
    Prob d{};
    d.P = p->n_poses;
    d.L = p->n_points;
    d.E = p->n_edges;
    d.n_cams = p->n_cams;
    d.cam_model = p->cam_model;
    d.delta = p->huber_delta;
    d.edge_point = p->edge_point;
    d.edge_pose = p->edge_pose;
    d.edge_obs = p->edge_obs;
    d.edge_w = p->edge_inv_sigma2;
    d.active = p->edge_active;
    d.cams = p->cams;
    d.pose_cam = p->pose_cam;
    d.pose_fixed = p->pose_fixed;
    d.pose_q = p->pose_q;
    d.pose_t = p->pose_t;
    d.point_xyz = p->point_xyz;
    return d;
}

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
    // gfx950: 160 KB of LDS per workgroup, less the factorization's static LDS; fall back to the 64 KB default if the
    // opt-in is refused
    c->ldlt_lds_budget = 0;
    hipFuncAttributes fa{};
    size_t stat = 8192;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&mam::lba::k_ldlt_any<true>)) == hipSuccess)
        stat = (fa.sharedSizeBytes + 255) / 256 * 256 + 256;
    else
        (void)hipGetLastError();
    // MAM_LBA_LDS_KB=<k> caps the budget (experiments: a factorization that leaves room on its CU for other work)
    size_t cap_kb = 160;
    if (const char* lk = std::getenv("MAM_LBA_LDS_KB")) cap_kb = std::max<size_t>(16, std::min<size_t>(160, (size_t)atoi(lk)));
    for (size_t budget : {cap_kb * 1024 - stat, (size_t)64 * 1024 - stat}) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::lba::k_ldlt_any<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)budget) == hipSuccess &&
            hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::lba::k_ldlt_any<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)budget) == hipSuccess &&
            hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::lba::k_ldlt_reg),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)budget) == hipSuccess &&
            hipFuncSetAttribute(reinterpret_cast<const void*>(&mam::lba::k_ldlt_mw),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)budget) == hipSuccess) {
            c->ldlt_lds_budget = budget;
            break;
        }
        (void)hipGetLastError();
    }
    // Highest stream priority: LocalMapping's solve shares the GPU with Tracking's full-chip launches, and its small
    // latency-bound kernels should not queue behind them. MAM_LBA_PRIORITY=0 keeps the default priority.
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
    for (auto& st : c->gstream)
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    for (auto& e : c->ev_done)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->up_stream) {
        (void)hipStreamSynchronize(c->up_stream);
        (void)hipStreamDestroy(c->up_stream);
    }
    if (c->up_done) (void)hipEventDestroy(c->up_done);
    delete c;
}

int mam_lba_set_cu_mask(mam_lba_ctx* c, int n_words, const uint32_t* mask) {
    if (!c || n_words < 0 || (n_words > 0 && !mask)) return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    // the group streams are re-created on the new mask at the next split batch
    for (int g = 0; g < mam_lba_ctx::kMaxGroups - 1; g++) {
        if (c->gstream[g]) {
            MAM_HIP(hipStreamSynchronize(c->gstream[g]));
            MAM_HIP(hipStreamDestroy(c->gstream[g]));
            c->gstream[g] = nullptr;
        }
        if (c->ev_done[g]) {
            MAM_HIP(hipEventDestroy(c->ev_done[g]));
            c->ev_done[g] = nullptr;
        }
    }
    c->cu_mask.assign(mask, mask + n_words);
    return MAM_OK;
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
    if (!c || !problem_ok(p) || !r || (p->n_poses > 0 && !p->pose_id) || (p->n_points > 0 && !p->point_id) ||
        !r->pose_q || !r->pose_t || (p->n_points > 0 && !r->point_xyz))
        return MAM_ERR_ARG;
    const int P = p->n_poses, L = p->n_points, E = p->n_edges;
    for (int e = 0; e < E; e++)
        if (p->edge_point[e] < 0 || p->edge_point[e] >= L || p->edge_pose[e] < 0 || p->edge_pose[e] >= P)
            return MAM_ERR_ARG;
    MAM_DEVICE_SCOPE(c->device);
    // g2o's Hessian order = vertices sorted by id (sparse_optimizer.cpp:166-190): the device path takes id-ordered
    // poses and points, so permute here and map the results back
    // (ids already ascending, as a window built in id order hands them over: identity, no sort)
    std::vector<int> po(P), pl(L), ipo(P), ipl(L);
    std::iota(po.begin(), po.end(), 0);
    std::iota(pl.begin(), pl.end(), 0);
    if (!std::is_sorted(p->pose_id, p->pose_id + P))
        std::stable_sort(po.begin(), po.end(), [&](int a, int b) { return p->pose_id[a] < p->pose_id[b]; });
    if (!std::is_sorted(p->point_id, p->point_id + L))
        std::stable_sort(pl.begin(), pl.end(), [&](int a, int b) { return p->point_id[a] < p->point_id[b]; });
    for (int i = 0; i < P; i++) ipo[po[i]] = i;
    for (int i = 0; i < L; i++) ipl[pl[i]] = i;
    bool ident_po = true, ident_pl = true;
    for (int i = 0; i < P && ident_po; i++) ident_po = po[i] == i;
    for (int i = 0; i < L && ident_pl; i++) ident_pl = pl[i] == i;
    int Np = 0;
    for (int i = 0; i < P; i++) Np += p->pose_fixed[i] ? 0 : 1;
    const int ncw = (p->cam_model == MAM_CAM_KANNALA_BRANDT8 ? 8 : 4) * p->n_cams;
    // staging layout (one H2D copy): inputs, then room for the outputs
    const size_t in_bytes = al(4 * (size_t)E) * 2 + al(16 * (size_t)E) + al(8 * (size_t)E) + al((size_t)E) +
                            al(4 * (size_t)ncw) + al(4 * (size_t)P) + al((size_t)P) + al(32 * (size_t)P) +
                            al(24 * (size_t)P) + al(24 * (size_t)L);
    const size_t out_bytes = al(32 * (size_t)P) + al(24 * (size_t)P) + al(24 * (size_t)L) + al(8 * (size_t)E) +
                             al((size_t)E);
    if (int rc = c->staging.alloc(in_bytes + out_bytes)) return rc;
    if (int rc = c->io.alloc(in_bytes + out_bytes)) return rc;
    uint8_t* hb = c->staging.p;
    Carver dv{c->io.p};
    auto put = [&](auto* dst_host_typed, size_t count) {
        using T = std::remove_pointer_t<decltype(dst_host_typed)>;
        T* d = dv.take<T>(count);
        return std::make_pair(d, reinterpret_cast<T*>(hb + (reinterpret_cast<uint8_t*>(d) - c->io.p)));
    };
    // two upload parts: what the structure build reads (edges' vertices, poses, points), then the observations and
    // their weights (read first by the linearisation), staged and copied while the GPU builds the structure
    auto [d_ep, h_ep] = put((int32_t*)nullptr, E);
    auto [d_eo, h_eo] = put((int32_t*)nullptr, E);
    auto [d_act, h_act] = put((uint8_t*)nullptr, E);
    auto [d_cams, h_cams] = put((float*)nullptr, ncw);
    auto [d_pc, h_pc] = put((int32_t*)nullptr, P);
    auto [d_fix, h_fix] = put((uint8_t*)nullptr, P);
    auto [d_q, h_q] = put((double*)nullptr, 4 * (size_t)P);
    auto [d_t, h_t] = put((double*)nullptr, 3 * (size_t)P);
    auto [d_x, h_x] = put((double*)nullptr, 3 * (size_t)L);
    const size_t upload_a = dv.off;
    auto [d_obs, h_obs] = put((double*)nullptr, 2 * (size_t)E);
    auto [d_w, h_w] = put((double*)nullptr, E);
    const size_t upload = dv.off;
    // staging: plain copies when the ids are already in Hessian order, permuted copies otherwise
    if (E) {
        if (ident_pl) std::memcpy(h_ep, p->edge_point, sizeof(int32_t) * E);
        else for (int e = 0; e < E; e++) h_ep[e] = ipl[p->edge_point[e]];
        if (ident_po) std::memcpy(h_eo, p->edge_pose, sizeof(int32_t) * E);
        else for (int e = 0; e < E; e++) h_eo[e] = ipo[p->edge_pose[e]];
        if (p->edge_active) std::memcpy(h_act, p->edge_active, E);
    }
    std::memcpy(h_cams, p->cams, sizeof(float) * ncw);
    for (int i = 0; i < P; i++) {
        const int s = po[i];
        h_pc[i] = p->pose_cam ? p->pose_cam[s] : 0;
        h_fix[i] = p->pose_fixed[s];
        for (int k = 0; k < 4; k++) h_q[4 * i + k] = p->pose_q[4 * s + k];
        for (int k = 0; k < 3; k++) h_t[3 * i + k] = p->pose_t[3 * s + k];
    }
    if (L && ident_pl) std::memcpy(h_x, p->point_xyz, sizeof(double) * 3 * (size_t)L);
    else
        for (int i = 0; i < L; i++)
            for (int k = 0; k < 3; k++) h_x[3 * i + k] = p->point_xyz[3 * pl[i] + k];
    Outs o{};
    o.q = dv.take<double>(4 * (size_t)P);
    o.t = dv.take<double>(3 * (size_t)P);
    o.xyz = dv.take<double>(3 * (size_t)L);
    o.chi2 = r->edge_chi2 ? dv.take<double>(E) : nullptr;
    o.depth = r->edge_depth_ok ? dv.take<uint8_t>(E) : nullptr;
    hipStream_t s = c->stream;
    if (upload_a) MAM_HIP(hipMemcpyAsync(c->io.p, hb, upload_a, hipMemcpyHostToDevice, s));
    // part two, once the structure build is enqueued: host staging copy (overlapping the GPU's build), then its upload
    // on the upload stream, which the linearisation waits for
    double* const hobs = h_obs;   // (structured bindings cannot be captured in C++17)
    double* const hw = h_w;
    auto upload_b = [&, hobs, hw](int* rc) -> hipEvent_t {
        if (E) {
            std::memcpy(hobs, p->edge_obs, sizeof(double) * 2 * (size_t)E);
            std::memcpy(hw, p->edge_inv_sigma2, sizeof(double) * E);
        }
        if (upload == upload_a) return nullptr;
        if (!c->up_stream) {
            if (hipStreamCreateWithFlags(&c->up_stream, hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&c->up_done, hipEventDisableTiming) != hipSuccess) {
                mam::set_last_error("LBA upload stream");
                *rc = MAM_ERR_DEVICE;
                return nullptr;
            }
        }
        if (hipMemcpyAsync(c->io.p + upload_a, hb + upload_a, upload - upload_a, hipMemcpyHostToDevice, c->up_stream) !=
                hipSuccess ||
            hipEventRecord(c->up_done, c->up_stream) != hipSuccess) {
            mam::set_last_error("LBA observation upload");
            *rc = MAM_ERR_DEVICE;
            return nullptr;
        }
        return c->up_done;
    };
    mam_lba_problem pd = *p;
    pd.edge_point = d_ep;
    pd.edge_pose = d_eo;
    pd.edge_obs = d_obs;
    pd.edge_inv_sigma2 = d_w;
    pd.edge_active = p->edge_active ? d_act : nullptr;
    pd.cams = d_cams;
    pd.pose_cam = d_pc;
    pd.pose_fixed = d_fix;
    pd.pose_q = d_q;
    pd.pose_t = d_t;
    pd.point_xyz = d_x;
    std::vector<Prob> hp{desc_of(&pd)};
    hp[0].Np = Np;
    std::vector<LM> lm0(1);
    std::memset(lm0.data(), 0, sizeof(LM));
    lm0[0].iterations = p->iterations;
    std::vector<Outs> outs{o};
    if (int rc = run_batch(c, hp, lm0, outs, stop_flag, s, r, upload_b)) return rc;
    // results back to the caller's order: one D2H copy of the output region into the pinned staging block (pageable
    // destinations were one staged, synchronous copy each)
    if (dv.off > upload) MAM_HIP(hipMemcpyAsync(hb + upload, c->io.p + upload, dv.off - upload, hipMemcpyDeviceToHost, s));
    MAM_HIP(hipStreamSynchronize(s));
    auto host_of = [&](auto* dptr) {
        using T = std::remove_cv_t<std::remove_pointer_t<decltype(dptr)>>;
        return reinterpret_cast<const T*>(hb + (reinterpret_cast<const uint8_t*>(dptr) - c->io.p));
    };
    const double* q = host_of(o.q);
    const double* t = host_of(o.t);
    const double* x = host_of(o.xyz);
    const double* chi = o.chi2 ? host_of(o.chi2) : nullptr;
    const uint8_t* dep = o.depth ? host_of(o.depth) : nullptr;
    if (r->status < 0) return r->status;
    for (int i = 0; i < P; i++) {
        const int d = po[i];
        for (int k = 0; k < 4; k++) r->pose_q[4 * d + k] = q[4 * i + k];
        for (int k = 0; k < 3; k++) r->pose_t[3 * d + k] = t[3 * i + k];
    }
    if (L && ident_pl) std::memcpy(r->point_xyz, x, sizeof(double) * 3 * (size_t)L);
    else
        for (int i = 0; i < L; i++)
            for (int k = 0; k < 3; k++) r->point_xyz[3 * pl[i] + k] = x[3 * i + k];
    for (int e = 0; e < E; e++) {
        if (o.chi2 && !(p->edge_active && !p->edge_active[e])) r->edge_chi2[e] = chi[e];
        if (o.depth) r->edge_depth_ok[e] = dep[e];
    }
    return MAM_OK;
}

int mam_lba_solve_batch_device(mam_lba_ctx* c, int n_problems, const mam_lba_problem* problems,
                               mam_lba_result* results, void* stream) {
    if (!c || n_problems < 0 || (n_problems > 0 && (!problems || !results))) return MAM_ERR_ARG;
    if (n_problems == 0) return MAM_OK;
    MAM_DEVICE_SCOPE(c->device);
    std::vector<Prob> hp(n_problems);
    std::vector<LM> lm0(n_problems);
    std::vector<Outs> outs(n_problems);
    for (int q = 0; q < n_problems; q++) {
        const mam_lba_problem* p = problems + q;
        const mam_lba_result* r = results + q;
        if (!problem_ok(p) || !r->pose_q || !r->pose_t || (p->n_points > 0 && !r->point_xyz) ||
            p->n_opt_poses < 0 || p->n_opt_poses > p->n_poses)
            return MAM_ERR_ARG;
        hp[q] = desc_of(p);
        hp[q].Np = p->n_opt_poses;
        std::memset(&lm0[q], 0, sizeof(LM));
        lm0[q].iterations = p->iterations;
        outs[q] = Outs{r->pose_q, r->pose_t, r->point_xyz, r->edge_chi2, r->edge_depth_ok};
    }
    return run_batch(c, hp, lm0, outs, nullptr, stream ? (hipStream_t)stream : c->stream, results);
}

}  // extern "C"
