"""TEST INFRASTRUCTURE ONLY — an independent float64 restatement of LocalBundleAdjustment's Levenberg-Marquardt solve,
used by tests/test_lba_dense_xcheck.py to cross-check the C oracle (oracle/lba_oracle.cpp), which produced the
self-generated golden fixture tests/golden/lba.npz. Nothing in mam3slam_amd/ imports it.

Written from g2o's published semantics, not from the C oracle: the whole Hessian is assembled densely (no Schur
complement, no block structure) and solved with numpy's LU, so a regression in the oracle's Schur / LDL^T / ordering
code shows up as a disagreement here.

  EdgeSE3ProjectXYZ (src/OptimizableTypes.cpp:139-160): e = obs - project(T X), point Jacobian
      -projectJac(Xc) R, pose Jacobian -projectJac(Xc) [[0, z, -y, 1, 0, 0], [-z, 0, x, 0, 1, 0], [y, -x, 0, 0, 0, 1]]
  RobustKernelHuber (core/robust_kernel_impl.cpp:76-91): rho(e2) = e2 (e2 <= d^2) else 2 d sqrt(e2) - d^2, and
      H += J^T rho' Omega J, b -= J^T rho' Omega e (core/base_binary_edge.hpp:54-120)
  SE3Quat exp / product (types/se3quat.h): T <- exp(dx) T, dx = (omega, upsilon)
  OptimizationAlgorithmLevenberg::solve (core/optimization_algorithm_levenberg.cpp:61-169), with ORB-SLAM3's
      stop rule ((iniChi - currentChi) 1e3 < iniChi three times in a row) and lambda_0 = 1e-5 max diag(H)

Pinhole cameras only (cam_model 0).
"""
from __future__ import annotations

import numpy as np


def _rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def _quat(R):
    """Unit quaternion (x, y, z, w) of a rotation matrix (Shepperd's method)."""
    tr = np.trace(R)
    if tr > 0:
        s = np.sqrt(tr + 1.0) * 2
        q = [(R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s, 0.25 * s]
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(1.0 + R[i, i] - R[j, j] - R[k, k]) * 2
        q = [0.0, 0.0, 0.0, (R[k, j] - R[j, k]) / s]
        q[i] = 0.25 * s
        q[j] = (R[j, i] + R[i, j]) / s
        q[k] = (R[k, i] + R[i, k]) / s
    return np.array(q)


def _qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz])


def _normalize(q):
    q = q / np.linalg.norm(q)
    return -q if q[3] < 0 else q


def _skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def se3_exp_mul(dx, q, t):
    """exp(dx) * (q, t), dx = (omega, upsilon)."""
    w, u = dx[:3], dx[3:]
    th = np.linalg.norm(w)
    O = _skew(w)
    O2 = O @ O
    if th < 1e-5:
        R = np.eye(3) + O + O2
        V = R
    else:
        R = np.eye(3) + np.sin(th) / th * O + (1 - np.cos(th)) / th ** 2 * O2
        V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * O + (th - np.sin(th)) / th ** 3 * O2
    qe = _normalize(_quat(R))
    return _normalize(_qmul(qe, q)), _rot(qe) @ t + V @ u


def _huber(e2, d):
    if d <= 0 or e2 <= d * d:
        return e2, 1.0
    s = np.sqrt(e2)
    return 2 * s * d - d * d, d / s


def solve(prob):
    """Returns dict(pose_q, pose_t, point_xyz, iterations, lm_trials) for an LBAProblem (Pinhole)."""
    assert int(prob.cam_model) == 0, "Pinhole only"
    P, L = len(prob.pose_id), len(prob.point_id)
    q = np.array([_normalize(np.asarray(x, np.float64)) for x in prob.pose_q])
    t = np.array(prob.pose_t, np.float64).copy()
    X = np.array(prob.point_xyz, np.float64).copy()
    fixed = np.asarray(prob.pose_fixed).astype(bool)
    hp = -np.ones(P, int)
    hp[~fixed] = np.arange(int((~fixed).sum()))   # Hessian pose block of each optimised pose (id order)
    Np = int((~fixed).sum())
    n = 6 * Np + 3 * L
    cams = np.asarray(prob.cams, np.float32).astype(np.float64)
    pc = np.zeros(P, int) if prob.pose_cam is None else np.asarray(prob.pose_cam)
    ep, epo = np.asarray(prob.edge_point), np.asarray(prob.edge_pose)
    obs, w = np.asarray(prob.edge_obs, np.float64), np.asarray(prob.edge_inv_sigma2, np.float64)
    act = np.ones(len(ep), bool) if prob.edge_active is None else np.asarray(prob.edge_active).astype(bool)
    delta = float(prob.huber_delta)

    def errors(q, t, X):
        es, xcs = [], []
        for k in range(len(ep)):
            i, p = epo[k], ep[k]
            Xc = _rot(q[i]) @ X[p] + t[i]
            fx, fy, cx, cy = cams[pc[i]][:4]
            es.append(obs[k] - np.array([fx * Xc[0] / Xc[2] + cx, fy * Xc[1] / Xc[2] + cy]))
            xcs.append(Xc)
        return es, xcs

    def chi(es):
        return sum(_huber(float(e @ e) * w[k], delta)[0] for k, e in enumerate(es) if act[k])

    def system(q, t, X):
        es, xcs = errors(q, t, X)
        H = np.zeros((n, n))
        b = np.zeros(n)
        for k in range(len(ep)):
            if not act[k]:
                continue
            i, p = epo[k], ep[k]
            x, y, z = xcs[k]
            fx, fy = cams[pc[i]][:2]
            Jp = -np.array([[fx / z, 0, -fx * x / z ** 2], [0, fy / z, -fy * y / z ** 2]])
            J = np.zeros((2, n))
            J[:, 6 * Np + 3 * p:6 * Np + 3 * p + 3] = Jp @ _rot(q[i])
            if hp[i] >= 0:
                D = np.array([[0, z, -y, 1, 0, 0], [-z, 0, x, 0, 1, 0], [y, -x, 0, 0, 0, 1]])
                J[:, 6 * hp[i]:6 * hp[i] + 6] = Jp @ D
            _, r1 = _huber(float(es[k] @ es[k]) * w[k], delta)
            H += J.T @ J * (r1 * w[k])
            b -= J.T @ es[k] * (r1 * w[k])
        return H, b, chi(es)

    def apply(dx):
        q2, t2 = q.copy(), t.copy()
        for i in range(P):
            if hp[i] >= 0:
                q2[i], t2[i] = se3_exp_mul(dx[6 * hp[i]:6 * hp[i] + 6], q[i], t[i])
        return q2, t2, X + dx[6 * Np:].reshape(L, 3)

    its = trials = 0
    if n == 0 or prob.iterations <= 0:
        return dict(pose_q=q, pose_t=t, point_xyz=X, iterations=0, lm_trials=0)
    lam, ni, nbad = 0.0, 2.0, 0
    for it in range(prob.iterations):
        H, b, cur = system(q, t, X)
        ini = cur
        if it == 0:
            lam, ni, nbad = 1e-5 * float(np.max(np.abs(np.diag(H)))), 2.0, 0
        qmax = 0
        while True:
            dx = np.linalg.solve(H + lam * np.eye(n), b)
            q2, t2, X2 = apply(dx)
            tmp = chi(errors(q2, t2, X2)[0])
            rho = (cur - tmp) / (float(dx @ (lam * dx + b)) + 1e-3)
            if rho > 0 and np.isfinite(tmp):
                alpha = min(1.0 - (2 * rho - 1) ** 3, 2.0 / 3.0)
                lam *= max(1.0 / 3.0, alpha)
                ni = 2.0
                cur = tmp
                q, t, X = q2, t2, X2
            else:
                lam *= ni
                ni *= 2
            qmax += 1
            trials += 1
            if not (rho < 0 and qmax < 10):
                break
        its += 1
        if qmax == 10 or rho == 0:
            break
        nbad = nbad + 1 if (ini - cur) * 1e3 < ini else 0
        if nbad >= 3:
            break
    return dict(pose_q=q, pose_t=t, point_xyz=X, iterations=its, lm_trials=trials)
