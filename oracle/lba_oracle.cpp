// lba_oracle.cpp — TEST INFRASTRUCTURE ONLY (see orb_oracle.h header note).
//
// Single-threaded FP64 CPU restatement of the g2o solve inside Optimizer::LocalBundleAdjustment
// (reference src/Optimizer.cc:1188-1410) with the vendored g2o it drives, step by step:
//   core/sparse_optimizer.cpp:166-190  buildIndexMapping (non-fixed poses by id, then points by id)
//   core/sparse_optimizer.cpp:355-436  optimize / update (oplus in _ivMap order)
//   core/sparse_optimizer.cpp:61-114   computeActiveErrors / activeRobustChi2 (edge insertion order)
//   core/optimization_algorithm_levenberg.cpp:61-194  LM trials, lambda init/update, scale, termination
//   core/block_solver.hpp:353-604      Schur complement, back-substitution, setLambda / restoreDiagonal
//   core/base_binary_edge.hpp:54-120   constructQuadraticForm (robust branch)
//   core/robust_kernel_impl.cpp:76-91  Huber
//   types/se3quat.h                    SE3Quat exp / map / product / normalizeRotation
//   src/OptimizableTypes.{h:99-110, cpp:139-160}  EdgeSE3ProjectXYZ error / Jacobians
//   src/CameraModels/Pinhole.cpp:35-41, 71-81      project / projectJac (float parameters)
// Eigen's SimplicialLDLT with AMD ordering is replaced by an envelope LDL^T of the reduced camera system (the sparse
// factorization's cost class, the same non-zeros + fill on banded covisibility) with the same failure rule (exact
// zero pivot); the difference is summation order only.

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>

#include "../include/mam_lba.h"
#include "../include/mam_orb.h"
#include "g2o_se3.h"
#include "../mam3slam_amd/csrc/camera.hpp"

namespace {

using namespace oracle_g2o;

struct Graph {
    const mam_lba_problem* p;
    std::vector<SE3> pose;
    std::vector<double> pt;                // 3 per point
    std::vector<int> pose_h;               // Hessian block of pose (-1 fixed)
    std::vector<int> point_h;              // Hessian block of point
    std::vector<int> hpose;                // inverse: Hessian pose block -> pose index
    std::vector<int> hpoint;
    int Np = 0, Nl = 0;
    // per-edge state
    std::vector<double> err;               // 2 per edge (last computeActiveErrors)
    // system
    std::vector<double> Hpp;               // 36 per Hessian pose
    std::vector<double> Hll;               // 9 per point
    std::vector<double> Hpl;               // 18 per edge: pose x landmark (6x3), row-major
    std::vector<double> b;                 // 6 Np + 3 Nl
    std::vector<double> x;

    bool kb8() const { return p->cam_model == MAM_CAM_KANNALA_BRANDT8; }
    const float* cam(int pose_idx) const {
        const int c = p->pose_cam ? p->pose_cam[pose_idx] : 0;
        return p->cams + (kb8() ? 8 : 4) * c;
    }
    // pCamera of an edge as a mam_camera (KannalaBrandt8: mvParameters fx, fy, cx, cy, k0..k3)
    mam_camera camera(int pose_idx) const {
        const float* c = cam(pose_idx);
        mam_camera m{};
        m.fx = c[0]; m.fy = c[1]; m.cx = c[2]; m.cy = c[3];
        if (kb8()) {
            for (int k = 0; k < 4; k++) m.k[k] = c[4 + k];
            m.model = MAM_CAM_KANNALA_BRANDT8;
        }
        return m;
    }

    void computeActiveErrors() {
        for (int e = 0; e < p->n_edges; e++) {
            const int ip = p->edge_pose[e], il = p->edge_point[e];
            double Xc[3];
            se3Map(pose[ip], &pt[3 * il], Xc);
            const float* c = cam(ip);
            double u, v;
            if (kb8()) {
                mam::cam::project_d(camera(ip), Xc, &u, &v);   // KannalaBrandt8::project(Vector3d) :46-65
            } else {
                u = c[0] * Xc[0] / Xc[2] + c[2];
                v = c[1] * Xc[1] / Xc[2] + c[3];
            }
            err[2 * e] = p->edge_obs[2 * e] - u;
            err[2 * e + 1] = p->edge_obs[2 * e + 1] - v;
        }
    }
    double chi2(int e) const {
        const double w = p->edge_inv_sigma2[e];
        const double e0 = err[2 * e], e1 = err[2 * e + 1];
        return e0 * (w * e0) + e1 * (w * e1);
    }
    bool active(int e) const { return !p->edge_active || p->edge_active[e]; }   // level 0
    void robustify(double e, double rho[3]) const {
        const double delta = p->huber_delta, dsqr = delta * delta;
        if (delta <= 0.0 || e <= dsqr) { rho[0] = e; rho[1] = 1.; rho[2] = 0.; }   // no kernel: rho(e) = e
        else {
            const double sqrte = std::sqrt(e);
            rho[0] = 2 * sqrte * delta - dsqr;
            rho[1] = delta / sqrte;
            rho[2] = -0.5 * rho[1] / e;
        }
    }
    double activeRobustChi2() const {
        double chi = 0.0, rho[3];
        for (int e = 0; e < p->n_edges; e++) {
            if (!active(e)) continue;
            robustify(chi2(e), rho);
            chi += rho[0];
        }
        return chi;
    }

    void buildSystem() {
        std::fill(Hpp.begin(), Hpp.end(), 0.0);
        std::fill(Hll.begin(), Hll.end(), 0.0);
        std::fill(Hpl.begin(), Hpl.end(), 0.0);
        std::fill(b.begin(), b.end(), 0.0);
        for (int e = 0; e < p->n_edges; e++) {
            if (!active(e)) continue;
            const int ip = p->edge_pose[e], il = p->edge_point[e];
            const SE3& T = pose[ip];
            double Xc[3];
            se3Map(T, &pt[3 * il], Xc);
            const double x = Xc[0], y = Xc[1], z = Xc[2];
            const float* c = cam(ip);
            // -projectJac (Pinhole.cpp:71-81 / KannalaBrandt8.cpp:145-175)
            double J[6] = {-(c[0] / z), -0.0, -(-c[0] * x / (z * z)), -0.0, -(c[1] / z), -(-c[1] * y / (z * z))};
            if (kb8()) {
                mam::cam::project_jac_d(camera(ip), Xc, J);
                for (int k = 0; k < 6; k++) J[k] = -J[k];
            }
            double R[9];
            toRotationMatrix(T.r, R);
            double A[6];   // 2x3 jacobianOplusXi = J R
            for (int r = 0; r < 2; r++)
                for (int k = 0; k < 3; k++)
                    A[3 * r + k] = J[3 * r] * R[k] + J[3 * r + 1] * R[3 + k] + J[3 * r + 2] * R[6 + k];
            const double D[18] = {0.0, z, -y, 1.0, 0.0, 0.0, -z, 0.0, x, 0.0, 1.0, 0.0, y, -x, 0.0, 0.0, 0.0, 1.0};
            double B[12];  // 2x6 jacobianOplusXj = J * SE3deriv
            for (int r = 0; r < 2; r++)
                for (int k = 0; k < 6; k++)
                    B[6 * r + k] = J[3 * r] * D[k] + J[3 * r + 1] * D[6 + k] + J[3 * r + 2] * D[12 + k];
            // robust branch of constructQuadraticForm
            const double w = p->edge_inv_sigma2[e];
            double rho[3];
            robustify(chi2(e), rho);
            const double orr[2] = {-(w * err[2 * e]) * rho[1], -(w * err[2 * e + 1]) * rho[1]};
            const double wo = rho[1] * w;   // weightedOmega = rho1 * invSigma2 * I
            const int hl = point_h[il];
            double* bl = &b[6 * Np + 3 * hl];
            double* Hl = &Hll[9 * hl];
            for (int i = 0; i < 3; i++) {
                bl[i] += A[i] * orr[0] + A[3 + i] * orr[1];
                for (int j = 0; j < 3; j++) Hl[3 * i + j] += A[i] * wo * A[j] + A[3 + i] * wo * A[3 + j];
            }
            const int hp = pose_h[ip];
            if (hp >= 0) {
                double* He = &Hpl[18 * e];   // pose x landmark = B^T W A
                for (int i = 0; i < 6; i++)
                    for (int j = 0; j < 3; j++) He[3 * i + j] += B[i] * wo * A[j] + B[6 + i] * wo * A[3 + j];
                double* bp = &b[6 * hp];
                double* Hp = &Hpp[36 * hp];
                for (int i = 0; i < 6; i++) {
                    bp[i] += B[i] * orr[0] + B[6 + i] * orr[1];
                    for (int j = 0; j < 6; j++) Hp[6 * i + j] += B[i] * wo * B[j] + B[6 + i] * wo * B[6 + j];
                }
            }
        }
    }

    double computeLambdaInit() const {
        double maxDiagonal = 0.;
        for (int h = 0; h < Np; h++)
            for (int j = 0; j < 6; j++) maxDiagonal = std::max(std::fabs(Hpp[36 * h + 7 * j]), maxDiagonal);
        for (int h = 0; h < Nl; h++)
            for (int j = 0; j < 3; j++) maxDiagonal = std::max(std::fabs(Hll[9 * h + 4 * j]), maxDiagonal);
        return 1e-5 * maxDiagonal;
    }

    static bool inv3(const double m[9], double o[9]) {
        // Eigen 3.4 compute_inverse<3> (LU/InverseImpl.h): the column-0 cofactors, det = their dot with column 0
        // summed c0 m00 + (c1 m10 + c2 m20) (the unrolled redux of a 3-vector, as camera.hpp inv3), invdet = 1 / det, result(r, c) = cofactor(c, r) * invdet
        const double c00 = m[4] * m[8] - m[5] * m[7], c10 = m[7] * m[2] - m[8] * m[1], c20 = m[1] * m[5] - m[2] * m[4];
        const double det = c00 * m[0] + (c10 * m[3] + c20 * m[6]);
        const double inv = 1.0 / det;
        o[0] = c00 * inv; o[1] = c10 * inv; o[2] = c20 * inv;
        o[3] = (m[5] * m[6] - m[3] * m[8]) * inv; o[4] = (m[8] * m[0] - m[6] * m[2]) * inv;
        o[5] = (m[2] * m[3] - m[0] * m[5]) * inv;
        o[6] = (m[3] * m[7] - m[4] * m[6]) * inv; o[7] = (m[6] * m[1] - m[7] * m[0]) * inv;
        o[8] = (m[0] * m[4] - m[1] * m[3]) * inv;
        return true;
    }

    // BlockSolver::setLambda + solve (Schur) + restoreDiagonal
    bool solve(double lambda, const std::vector<std::vector<int>>& point_edges) {
        const int n = 6 * Np;
        std::vector<double> S((size_t)n * n, 0.0), bs(n);
        for (int h = 0; h < Np; h++)
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 6; j++) S[(size_t)(6 * h + i) * n + 6 * h + j] = Hpp[36 * h + 6 * i + j] + (i == j ? lambda : 0.0);
        std::vector<double> coeff(n, 0.0), Dinv(9 * (size_t)Nl);
        for (int hl = 0; hl < Nl; hl++) {
            const int il = hpoint[hl];
            double D[9];
            for (int k = 0; k < 9; k++) D[k] = Hll[9 * hl + k] + ((k % 4 == 0) ? lambda : 0.0);
            double* Di = &Dinv[9 * (size_t)hl];
            inv3(D, Di);
            const double* bl = &b[n + 3 * hl];
            double db[3];
            for (int i = 0; i < 3; i++) db[i] = Di[3 * i] * bl[0] + Di[3 * i + 1] * bl[1] + Di[3 * i + 2] * bl[2];
            const std::vector<int>& E = point_edges[il];
            for (size_t a = 0; a < E.size(); a++) {
                const int ea = E[a], ha = pose_h[p->edge_pose[ea]];
                if (ha < 0) continue;
                const double* Ba = &Hpl[18 * (size_t)ea];
                double BDinv[18];
                for (int i = 0; i < 6; i++)
                    for (int j = 0; j < 3; j++)
                        BDinv[3 * i + j] = Ba[3 * i] * Di[j] + Ba[3 * i + 1] * Di[3 + j] + Ba[3 * i + 2] * Di[6 + j];
                for (int i = 0; i < 6; i++) coeff[6 * ha + i] += Ba[3 * i] * db[0] + Ba[3 * i + 1] * db[1] + Ba[3 * i + 2] * db[2];
                for (size_t c = 0; c < E.size(); c++) {
                    const int ec = E[c], hc = pose_h[p->edge_pose[ec]];
                    if (hc < 0 || hc < ha) continue;   // upper blocks (i2 >= i1)
                    const double* Bc = &Hpl[18 * (size_t)ec];
                    for (int i = 0; i < 6; i++)
                        for (int j = 0; j < 6; j++)
                            S[(size_t)(6 * ha + i) * n + 6 * hc + j] -=
                                BDinv[3 * i] * Bc[3 * j] + BDinv[3 * i + 1] * Bc[3 * j + 1] + BDinv[3 * i + 2] * Bc[3 * j + 2];
                }
            }
        }
        for (int i = 0; i < n; i++) bs[i] = b[i] - coeff[i];
        // LDL^T of the symmetric reduced system on its envelope (profile): Eigen's SimplicialLDLT factors the sparse
        // reduced system, whose non-zeros (pose blocks sharing a landmark) and fill lie inside the envelope of the
        // block rows — the same cost class (n b^2 on a window's banded covisibility), not a dense n^3 / 6 (which
        // overstated the reference's factorization ~7x at 50 keyframes). Row i's envelope starts at f[i]: the first
        // pose block sharing a landmark with i's block. Same failure rule (an exact zero pivot).
        for (int i = 0; i < n; i++)
            for (int j = 0; j < i; j++) S[(size_t)i * n + j] = S[(size_t)j * n + i];
        std::vector<int> fblk(Np);
        for (int h = 0; h < Np; h++) fblk[h] = h;
        for (int hl = 0; hl < Nl; hl++) {
            int mn = Np;
            for (int e : point_edges[hpoint[hl]]) {
                const int h = pose_h[p->edge_pose[e]];
                if (h >= 0) mn = std::min(mn, h);
            }
            for (int e : point_edges[hpoint[hl]]) {
                const int h = pose_h[p->edge_pose[e]];
                if (h >= 0) fblk[h] = std::min(fblk[h], mn);
            }
        }
        std::vector<int> f(n);
        for (int i = 0; i < n; i++) f[i] = 6 * fblk[i / 6];
        std::vector<double> L((size_t)n * n, 0.0), d(n);
        for (int i = 0; i < n; i++) {
            const int fi = f[i];
            double* Li = &L[(size_t)i * n];
            for (int j = fi; j < i; j++) {
                const double* Lj = &L[(size_t)j * n];
                double t = S[(size_t)i * n + j];
                for (int k = std::max(fi, f[j]); k < j; k++) t -= Li[k] * Lj[k] * d[k];
                Li[j] = t / d[j];
            }
            double sd = S[(size_t)i * n + i];
            for (int k = fi; k < i; k++) sd -= Li[k] * Li[k] * d[k];
            if (sd == 0.0) return false;
            d[i] = sd;
        }
        std::vector<double> yv(n);
        for (int i = 0; i < n; i++) {
            double t = bs[i];
            for (int k = f[i]; k < i; k++) t -= L[(size_t)i * n + k] * yv[k];
            yv[i] = t;
        }
        for (int i = 0; i < n; i++) x[i] = yv[i] / d[i];
        for (int k = n - 1; k >= 0; k--)
            for (int i = f[k]; i < k; i++) x[i] -= L[(size_t)k * n + i] * x[k];
        // landmarks: xl = Dinv (bl - Hpl^T xp)
        for (int hl = 0; hl < Nl; hl++) {
            const int il = hpoint[hl];
            double cl[3] = {b[n + 3 * hl], b[n + 3 * hl + 1], b[n + 3 * hl + 2]};
            for (int e : point_edges[il]) {
                const int h = pose_h[p->edge_pose[e]];
                if (h < 0) continue;
                const double* Be = &Hpl[18 * (size_t)e];
                for (int j = 0; j < 3; j++)
                    for (int i = 0; i < 6; i++) cl[j] -= Be[3 * i + j] * x[6 * h + i];
            }
            const double* Di = &Dinv[9 * (size_t)hl];
            for (int i = 0; i < 3; i++) x[n + 3 * hl + i] = Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1] + Di[3 * i + 2] * cl[2];
        }
        return true;
    }

    void update() {
        for (int h = 0; h < Np; h++) {
            const int ip = hpose[h];
            pose[ip] = se3Mul(se3Exp(&x[6 * h]), pose[ip]);
        }
        for (int hl = 0; hl < Nl; hl++) {
            const int il = hpoint[hl];
            for (int i = 0; i < 3; i++) pt[3 * il + i] += x[6 * Np + 3 * hl + i];
        }
    }

    double computeScale(double lambda) const {
        double scale = 0.;
        for (size_t j = 0; j < x.size(); j++) scale += x[j] * (lambda * x[j] + b[j]);
        return scale;
    }
};

}  // namespace

extern "C" int oracle_lba_solve(const mam_lba_problem* p, const volatile uint8_t* stop_flag, mam_lba_result* r) {
    if (!p || !r || p->n_poses < 0 || p->n_points < 0 || p->n_edges < 0) return MAM_ERR_ARG;
    Graph g;
    g.p = p;
    g.pose.resize(p->n_poses);
    for (int i = 0; i < p->n_poses; i++) {
        g.pose[i].r = {p->pose_q[4 * i], p->pose_q[4 * i + 1], p->pose_q[4 * i + 2], p->pose_q[4 * i + 3]};
        for (int k = 0; k < 3; k++) g.pose[i].t[k] = p->pose_t[3 * i + k];
        normalizeRotation(g.pose[i]);   // SE3Quat(q, t) constructor
    }
    g.pt.assign(p->point_xyz, p->point_xyz + 3 * (size_t)p->n_points);
    // _ivMap (sparse_optimizer.cpp:166-190): vertices sorted by id; non-fixed poses, then points
    std::vector<int> po(p->n_poses), pl(p->n_points);
    std::iota(po.begin(), po.end(), 0);
    std::iota(pl.begin(), pl.end(), 0);
    std::stable_sort(po.begin(), po.end(), [&](int a, int b) { return p->pose_id[a] < p->pose_id[b]; });
    std::stable_sort(pl.begin(), pl.end(), [&](int a, int b) { return p->point_id[a] < p->point_id[b]; });
    g.pose_h.assign(p->n_poses, -1);
    for (int i : po)
        if (!p->pose_fixed[i]) { g.pose_h[i] = g.Np++; g.hpose.push_back(i); }
    g.point_h.assign(p->n_points, -1);
    for (int i : pl) { g.point_h[i] = g.Nl++; g.hpoint.push_back(i); }
    std::vector<std::vector<int>> point_edges(p->n_points);
    for (int e = 0; e < p->n_edges; e++) point_edges[p->edge_point[e]].push_back(e);
    g.err.assign(2 * (size_t)p->n_edges, 0.0);
    g.Hpp.assign(36 * (size_t)g.Np, 0.0);
    g.Hll.assign(9 * (size_t)g.Nl, 0.0);
    g.Hpl.assign(18 * (size_t)p->n_edges, 0.0);
    g.b.assign(6 * (size_t)g.Np + 3 * (size_t)g.Nl, 0.0);
    g.x.assign(g.b.size(), 0.0);

    auto terminate = [&]() { return stop_flag && *stop_flag; };
    double currentLambda = -1.0, ni = 2.0;
    int nBad = 0, trials = 0, its = 0;
    int status = 0;
    g.computeActiveErrors();
    r->initial_chi2 = g.activeRobustChi2();
    bool ok = g.Np + g.Nl > 0;
    for (int it = 0; it < p->iterations && !terminate() && ok; it++) {
        g.computeActiveErrors();
        double currentChi = g.activeRobustChi2();
        const double iniChi = currentChi;
        g.buildSystem();
        if (it == 0) { currentLambda = g.computeLambdaInit(); ni = 2; nBad = 0; }
        double rho = 0;
        int qmax = 0;
        do {
            std::vector<SE3> bp = g.pose;   // push
            std::vector<double> bpt = g.pt;
            const bool ok2 = g.solve(currentLambda, point_edges);
            g.update();
            g.computeActiveErrors();
            double tempChi = g.activeRobustChi2();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = g.computeScale(currentLambda);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                currentLambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                currentLambda *= ni;
                ni *= 2;
                g.pose = bp;   // pop
                g.pt = bpt;
            }
            qmax++;
            trials++;
        } while (rho < 0 && qmax < 10 && !terminate());
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
    if (terminate()) status = 1;
    for (int i = 0; i < p->n_poses; i++) {
        r->pose_q[4 * i] = g.pose[i].r.x; r->pose_q[4 * i + 1] = g.pose[i].r.y;
        r->pose_q[4 * i + 2] = g.pose[i].r.z; r->pose_q[4 * i + 3] = g.pose[i].r.w;
        for (int k = 0; k < 3; k++) r->pose_t[3 * i + k] = g.pose[i].t[k];
    }
    memcpy(r->point_xyz, g.pt.data(), sizeof(double) * 3 * (size_t)p->n_points);
    // chi2() reads the error of the LAST computeActiveErrors (a rejected trial's, if the run ended on one);
    // isDepthPositive() recomputes from the current estimates (OptimizableTypes.h:99-110)
    for (int e = 0; e < p->n_edges; e++) {
        if (r->edge_chi2 && g.active(e)) r->edge_chi2[e] = g.chi2(e);
        if (r->edge_depth_ok) {
            double Xc[3];
            se3Map(g.pose[p->edge_pose[e]], &g.pt[3 * p->edge_point[e]], Xc);
            r->edge_depth_ok[e] = Xc[2] > 0.0;
        }
    }
    g.computeActiveErrors();
    r->final_chi2 = g.activeRobustChi2();
    r->iterations = its;
    r->lm_trials = trials;
    r->status = status;
    return MAM_OK;
}
