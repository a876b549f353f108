// pose_oracle.cpp — TEST INFRASTRUCTURE ONLY (see orb_oracle.h header note).
//
// Single-threaded FP64 CPU restatement of Optimizer::PoseOptimization for mono Pinhole frames (reference
// src/Optimizer.cc:814-1115) and the vendored g2o pieces it drives:
//   Optimizer.cc:856-895          one EdgeSE3ProjectXYZOnlyPose per matched keypoint, Huber(sqrt(5.991)), in
//                                 keypoint order; nInitialCorrespondences < 3 -> return 0 (:997-998)
//   Optimizer.cc:1001-1100        4 rounds: pose reset to the frame's pose, initializeOptimization(0), optimize(10),
//                                 chi2 > 5.991 -> outlier (level 1; outliers get computeError() first), robust
//                                 kernel dropped after round 2, stop early if fewer than 10 edges
//   core/sparse_optimizer.cpp:206-268, 355-420  active edges = level 0 (insertion order); no active edge -> no
//                                 optimisation (optimize returns -1)
//   core/optimization_algorithm_levenberg.cpp:61-194  LM trials, lambda init 1e-5 * max diag, scale, Raul's stop
//   core/base_unary_edge.hpp:43-71                    constructQuadraticForm (robust and plain branches)
//   core/robust_kernel_impl.cpp:76-91                 Huber
//   solvers/linear_solver_dense.h:65-118              Eigen LDLT<MatrixXd> (Lower) with diagonal pivoting and
//                                                     the pseudo-inverse of D in solve (Eigen 3.4.0 LDLT.h)
//   src/OptimizableTypes.{h:31-57, cpp:49-63}         error, isDepthPositive, Jacobian (-projectJac * SE3deriv)
//   src/CameraModels/Pinhole.cpp:35-41, 71-81         project / projectJac (float parameters)
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "../include/mam_pose.h"
#include "g2o_se3.h"
#include "../mam3slam_amd/csrc/camera.hpp"

namespace {

using namespace oracle_g2o;

struct PoseProblem {
    const mam_pinhole* cam;
    int n;
    const mam_pose_edge* e;
    std::vector<uint8_t> level;   // 0 active, 1 outlier
    std::vector<double> err;      // 2 per edge: last computeError()
    bool robust = true;
    double delta = (double)(float)std::sqrt(5.991);   // const float deltaMono (Optimizer.cc:850)

    void computeError(const SE3& T, int i) {
        const double X[3] = {(double)e[i].xw[0], (double)e[i].xw[1], (double)e[i].xw[2]};
        double Xc[3];
        se3Map(T, X, Xc);
        double u, v;
        if (cam->model == MAM_CAM_KANNALA_BRANDT8) {
            mam::cam::project_d(*cam, Xc, &u, &v);   // KannalaBrandt8::project(Vector3d)
        } else {
            u = (double)cam->fx * Xc[0] / Xc[2] + (double)cam->cx;
            v = (double)cam->fy * Xc[1] / Xc[2] + (double)cam->cy;
        }
        err[2 * i] = (double)e[i].obs[0] - u;
        err[2 * i + 1] = (double)e[i].obs[1] - v;
    }
    double chi2(int i) const {
        const double w = (double)e[i].inv_sigma2;
        const double e0 = err[2 * i], e1 = err[2 * i + 1];
        return e0 * (w * e0) + e1 * (w * e1);
    }
    void rho(double c, double r[3]) const {
        if (!robust) { r[0] = c; r[1] = 1.0; r[2] = 0.0; return; }
        const double dsqr = delta * delta;
        if (c <= dsqr) { r[0] = c; r[1] = 1.; r[2] = 0.; }
        else {
            const double sqrte = std::sqrt(c);
            r[0] = 2 * sqrte * delta - dsqr;
            r[1] = delta / sqrte;
            r[2] = -0.5 * r[1] / c;
        }
    }
    void computeActiveErrors(const SE3& T) {
        for (int i = 0; i < n; i++)
            if (!level[i]) computeError(T, i);
    }
    double activeRobustChi2() const {
        double chi = 0.0, r[3];
        for (int i = 0; i < n; i++) {
            if (level[i]) continue;
            rho(chi2(i), r);
            chi += r[0];
        }
        return chi;
    }
    // H (6x6, full) and b of the single pose vertex
    void buildSystem(const SE3& T, double H[36], double b[6]) const {
        std::fill(H, H + 36, 0.0);
        std::fill(b, b + 6, 0.0);
        for (int i = 0; i < n; i++) {
            if (level[i]) continue;
            const double X[3] = {(double)e[i].xw[0], (double)e[i].xw[1], (double)e[i].xw[2]};
            double Xc[3];
            se3Map(T, X, Xc);
            const double x = Xc[0], y = Xc[1], z = Xc[2];
            const double fx = cam->fx, fy = cam->fy;
            // -projectJac (Pinhole.cpp:71-81) * SE3deriv (OptimizableTypes.cpp:49-63)
            double J[6] = {-(fx / z), -0.0, -(-fx * x / (z * z)), -0.0, -(fy / z), -(-fy * y / (z * z))};
            if (cam->model == MAM_CAM_KANNALA_BRANDT8) {   // KannalaBrandt8::projectJac
                mam::cam::project_jac_d(*cam, Xc, J);
                for (int k = 0; k < 6; k++) J[k] = -J[k];
            }
            const double D[18] = {0.0, z, -y, 1.0, 0.0, 0.0, -z, 0.0, x, 0.0, 1.0, 0.0, y, -x, 0.0, 0.0, 0.0, 1.0};
            double A[12];
            for (int r = 0; r < 2; r++)
                for (int k = 0; k < 6; k++) A[6 * r + k] = J[3 * r] * D[k] + J[3 * r + 1] * D[6 + k] + J[3 * r + 2] * D[12 + k];
            const double w = (double)e[i].inv_sigma2;
            double r3[3];
            rho(chi2(i), r3);
            const double orr[2] = {-(w * err[2 * i]) * r3[1], -(w * err[2 * i + 1]) * r3[1]};
            const double wo = r3[1] * w;
            for (int a = 0; a < 6; a++) {
                b[a] += A[a] * orr[0] + A[6 + a] * orr[1];
                for (int c = 0; c < 6; c++) H[6 * a + c] += A[a] * wo * A[c] + A[6 + a] * wo * A[6 + c];
            }
        }
    }
};

// Eigen 3.4.0 LDLT<MatrixXd, Lower>::compute + solve on a 6x6 system. Returns isPositive().
bool eigen_ldlt_solve(const double Hin[36], const double bin[6], double x[6]) {
    const int n = 6;
    double m[36];
    std::memcpy(m, Hin, sizeof(m));
    int tr[6];
    double temp[6];
    enum { ZeroSign, PositiveSemiDef, NegativeSemiDef, Indefinite } sign = ZeroSign;
    bool found_zero_pivot = false;
    for (int k = 0; k < n; k++) {
        int big = k;
        double bv = std::fabs(m[7 * k]);
        for (int i = k + 1; i < n; i++)
            if (std::fabs(m[7 * i]) > bv) { bv = std::fabs(m[7 * i]); big = i; }   // maxCoeff: first maximum
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; j++) std::swap(m[6 * k + j], m[6 * big + j]);               // rows, head(k)
            for (int i = big + 1; i < n; i++) std::swap(m[6 * i + k], m[6 * i + big]);         // cols, tail(s)
            std::swap(m[7 * k], m[7 * big]);
            for (int i = k + 1; i < big; i++) {
                const double t = m[6 * i + k];
                m[6 * i + k] = m[6 * big + i];
                m[6 * big + i] = t;
            }
        }
        const int rs = n - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; j++) temp[j] = m[7 * j] * m[6 * k + j];
            double s = 0.0;
            for (int j = 0; j < k; j++) s += m[6 * k + j] * temp[j];
            m[7 * k] -= s;
            for (int i = k + 1; i < n; i++) {
                double t = 0.0;
                for (int j = 0; j < k; j++) t += m[6 * i + j] * temp[j];
                m[6 * i + k] -= t;
            }
        }
        const double akk = m[7 * k];
        const bool valid = std::fabs(akk) > 0.0;
        if (k == 0 && !valid) {   // the whole diagonal is zero
            sign = ZeroSign;
            for (int j = 0; j < n; j++) tr[j] = j;
            break;
        }
        if (rs > 0 && valid)
            for (int i = k + 1; i < n; i++) m[6 * i + k] /= akk;
        if (!valid) found_zero_pivot = true;
        if (sign == PositiveSemiDef) { if (akk < 0) sign = Indefinite; }
        else if (sign == NegativeSemiDef) { if (akk > 0) sign = Indefinite; }
        else if (sign == ZeroSign) { if (akk > 0) sign = PositiveSemiDef; else if (akk < 0) sign = NegativeSemiDef; }
    }
    (void)found_zero_pivot;
    // solve: P b, L^-1, D^+ (tolerance numeric_limits::min), L^-T, P^T
    double d[6];
    std::memcpy(d, bin, sizeof(d));
    for (int k = 0; k < n; k++) std::swap(d[k], d[tr[k]]);
    for (int k = 0; k < n; k++)
        for (int i = k + 1; i < n; i++) d[i] -= m[6 * i + k] * d[k];
    const double tol = std::numeric_limits<double>::min();
    for (int i = 0; i < n; i++) d[i] = std::fabs(m[7 * i]) > tol ? d[i] / m[7 * i] : 0.0;
    for (int k = n - 1; k >= 0; k--)
        for (int i = 0; i < k; i++) d[i] -= m[6 * k + i] * d[k];
    for (int k = n - 1; k >= 0; k--) std::swap(d[k], d[tr[k]]);
    std::memcpy(x, d, sizeof(d));
    return sign == PositiveSemiDef || sign == ZeroSign;
}

// SparseOptimizer::optimize(10) with OptimizationAlgorithmLevenberg on the single pose vertex. Returns the
// iterations run (0 when there is no active edge: optimize() returns -1 before the loop).
int optimize(PoseProblem& P, SE3& T, int iterations, int* trials_out) {
    bool any = false;
    for (int i = 0; i < P.n; i++) any = any || !P.level[i];
    if (!any) return 0;
    double lambda = 0.0, ni = 2.0;
    int nBad = 0, its = 0;
    bool ok = true;
    for (int it = 0; it < iterations && ok; it++) {
        P.computeActiveErrors(T);
        double currentChi = P.activeRobustChi2();
        const double iniChi = currentChi;
        double H[36], b[6];
        P.buildSystem(T, H, b);
        if (it == 0) {
            double md = 0.0;
            for (int j = 0; j < 6; j++) md = std::max(std::fabs(H[7 * j]), md);
            lambda = 1e-5 * md;
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            double Hl[36], x[6];
            std::memcpy(Hl, H, sizeof(Hl));
            for (int j = 0; j < 6; j++) Hl[7 * j] += lambda;
            const bool ok2 = eigen_ldlt_solve(Hl, b, x);
            const SE3 Tn = se3Mul(se3Exp(x), T);   // VertexSE3Expmap::oplusImpl
            P.computeActiveErrors(Tn);
            double tempChi = P.activeRobustChi2();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = 0.0;
            for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
                T = Tn;
            } else {
                lambda *= ni;
                ni *= 2;   // pop: T unchanged (the errors stay those of the rejected trial)
            }
            qmax++;
            (*trials_out)++;
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

}  // namespace

extern "C" int oracle_pose_optimization(const mam_pose* tcw, const mam_pinhole* cam, int n, const mam_pose_edge* edges,
                                        uint8_t* outlier, mam_pose_result* res) {
    if (!tcw || !cam || n < 0 || (n > 0 && (!edges || !outlier)) || !res) return MAM_ERR_ARG;
    SE3 T0;
    T0.r = {(double)tcw->q[0], (double)tcw->q[1], (double)tcw->q[2], (double)tcw->q[3]};
    for (int k = 0; k < 3; k++) T0.t[k] = (double)tcw->t[k];
    normalizeRotation(T0);   // SE3Quat(q, t)
    res->rounds = res->iterations = res->lm_trials = 0;
    for (int i = 0; i < n; i++) outlier[i] = 0;   // mvbOutlier[i] = false while the edges are added
    auto put = [&](const SE3& T) {
        res->q[0] = T.r.x; res->q[1] = T.r.y; res->q[2] = T.r.z; res->q[3] = T.r.w;
        for (int k = 0; k < 3; k++) res->t[k] = T.t[k];
    };
    if (n < 3) {
        put(T0);
        res->n_inliers = 0;
        return 0;
    }
    PoseProblem P;
    P.cam = cam;
    P.n = n;
    P.e = edges;
    P.level.assign(n, 0);
    P.err.assign(2 * (size_t)n, 0.0);
    SE3 T = T0;
    int nBad = 0;
    for (int it = 0; it < 4; it++) {
        T = T0;   // vSE3->setEstimate(pFrame->GetPose())
        res->iterations += optimize(P, T, 10, &res->lm_trials);
        res->rounds++;
        nBad = 0;
        for (int i = 0; i < n; i++) {
            if (outlier[i]) P.computeError(T, i);
            const float c = (float)P.chi2(i);   // const float chi2 = e->chi2() (Optimizer.cc:1025)
            if (c > 5.991f) {                   // chi2Mono[it]
                outlier[i] = 1;
                P.level[i] = 1;
                nBad++;
            } else {
                outlier[i] = 0;
                P.level[i] = 0;
            }
        }
        if (it == 2) P.robust = false;
        if (n < 10) break;
    }
    put(T);
    res->n_inliers = n - nBad;
    return res->n_inliers;
}
