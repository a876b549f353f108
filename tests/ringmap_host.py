"""Host restatement of the device map's LocalMapping edits (include/mam_ringmap.h, csrc/ringmap.hip) — TEST
INFRASTRUCTURE ONLY, the checker of tests/test_ringmap_gpu.py. Written from the rules the header states, which follow
src/LocalMapping.cc:457-501 (MapPointCulling), 504-828 (CreateNewMapPoints), 830-939 (SearchInNeighbors);
src/ORBmatcher.cc:1148-1338 (Fuse's Replace / AddObservation); src/MapPoint.cc:141-239, 248-297, 329-403, 426-494;
src/KeyFrame.cc:312-380 (UpdateConnections); src/Optimizer.cc:1118-1186, 1413-1497 (LocalBundleAdjustment's window and
write-back) — plain Python loops over numpy state, one MapPoint / keypoint at a time, in the reference's order where
the header fixes one.

State: dict(mp_of int32 [R S], okp int16 [R S][R], rec FUSE_MP_DTYPE [R S], born int32 [R S], tcw float32 [R][7]);
ring: dict(keys KP_DTYPE [R][S], desc uint8 [R][S][32], cnt int [R], kp_rec FUSE_MP_DTYPE [R S], sf float32 [L],
inv_s2 float32 [L])."""
from __future__ import annotations

import numpy as np

F32 = np.float32


def _obs(st, m):
    return [(s, int(k)) for s, k in enumerate(st["okp"][m]) if k >= 0]


def _set_bad(st, m):
    for s, k in _obs(st, m):
        st["mp_of"][s * st["S"] + k] = -1
    st["okp"][m][:] = -1
    st["rec"][m]["valid"] = 0


def _rehome(st, m):
    """Move MapPoint m to the keypoint of its lowest observing slot; returns the new id."""
    S = st["S"]
    s, k = _obs(st, m)[0]
    n = s * S + k
    st["okp"][n][:] = st["okp"][m]
    st["okp"][m][:] = -1
    for s2, k2 in _obs(st, n):
        st["mp_of"][s2 * S + k2] = n
    st["rec"][n] = st["rec"][m]
    st["born"][n] = st["born"][m]
    st["rec"][m]["valid"] = 0
    return n


def _repair(st, ids, bad_rule):
    """Decide for every live id first (bad / rehome / keep), then apply (the two device passes)."""
    S = st["S"]
    dec = {}
    for m in ids:
        if not st["rec"][m]["valid"]:
            continue
        n = len(_obs(st, m))
        if bad_rule(m, n) or n == 0:
            dec[m] = -2
        elif st["mp_of"][m] != m:
            s, k = _obs(st, m)[0]
            dec[m] = s * S + k
    newid = {}
    for m in sorted(dec):
        if dec[m] == -2:
            _set_bad(st, m)
            newid[m] = -1
        else:
            newid[m] = _rehome(st, m)
    return newid


def evict(st, head, W, run):
    """KeyFrame::SetBadFlag of slots [head, head + W) + MapPointCulling (mono nThObs 2)."""
    S, R = st["S"], st["R"]
    lost = set()
    for s in range(head, head + W):
        for k in range(S):
            m = st["mp_of"][s * S + k]
            if m >= 0:
                st["okp"][m][s] = -1
                st["mp_of"][s * S + k] = -1
                lost.add(int(m))
    _repair(st, range(R * S), lambda m, n: n <= 2 and (m in lost or st["born"][m] == run - 1))


def create(st, ring, head, W, pairs, NN, match, run):
    """CreateNewMapPoints: keypoint i1 takes its first neighbour match; the lowest (w, i1) claimant of a neighbour
    keypoint wins it."""
    S = st["S"]
    cnt = ring["cnt"]
    picks, claim = {}, {}
    for w in range(W):
        j = head + w
        for i1 in range(min(int(cnt[j]), S)):
            if st["mp_of"][j * S + i1] >= 0:
                continue
            for k in range(NN):
                nb = int(pairs[w * NN + k, 1])
                i2 = int(match[w * NN + k, i1])
                if 0 <= i2 < min(int(cnt[nb]), S) and st["mp_of"][nb * S + i2] < 0:
                    t = nb * S + i2
                    picks[(w, i1)] = t
                    key = w * S + i1
                    claim[t] = min(claim.get(t, key), key)
                    break
    for (w, i1), t in picks.items():
        if claim[t] != w * S + i1:
            continue
        j = head + w
        mid = j * S + i1
        r = ring["kp_rec"][mid].copy()
        r["valid"] = 1
        st["rec"][mid] = r
        st["born"][mid] = run
        st["mp_of"][mid] = mid
        st["mp_of"][t] = mid
        st["okp"][mid][j] = i1
        st["okp"][mid][t // S] = t % S


def gather(st):
    """Fuse's MapPoint lists (FUSE_MP_DTYPE [R S])."""
    out = np.zeros_like(st["rec"])
    for e, m in enumerate(st["mp_of"]):
        if m >= 0:
            out[e] = st["rec"][m]
            out[e]["valid"] = 1
    return out


def _proposals(st, ring, head, W, pairs, NN, NB, fwd, bwd):
    S = st["S"]
    cnt = ring["cnt"]
    out = []
    for b in range(W * NN):
        w = b // NN
        j, nb = head + w, int(pairs[b, 1])
        for i in range(min(int(cnt[j]), S)):
            idx = int(fwd[b, i])
            if idx < 0 or idx >= min(int(cnt[nb]), S):
                continue
            m = int(st["mp_of"][j * S + i])
            if m >= 0 and st["okp"][m][nb] < 0:
                out.append((m, nb * S + idx))
    for b in range(W * NB):
        w, k = b // NB, b % NB
        j = head + w
        nbk = int(pairs[w * NN + k, 1])
        for i in range(min(int(cnt[nbk]), S)):
            idx = int(bwd[b, i])
            if idx < 0 or idx >= min(int(cnt[j]), S):
                continue
            m = int(st["mp_of"][nbk * S + i])
            if m < 0:
                continue
            if any(st["okp"][m][int(pairs[w * NN + k2, 1])] >= 0 for k2 in range(k)):
                continue
            if st["okp"][m][j] < 0:
                out.append((m, j * S + idx))
    return out


def fuse_apply(st, ring, head, W, pairs, NN, NB, fwd, bwd):
    """Fuse's Replace / AddObservation over the run's proposals (components, survivors, one keypoint per keyframe)."""
    S, R = st["S"], st["R"]
    props = _proposals(st, ring, head, W, pairs, NN, NB, fwd, bwd)
    parent = {}

    def find(x):
        while parent.get(x, x) != x:
            x = parent[x]
        return x

    def union(a, b):
        a, b = find(a), find(b)
        if a != b:
            lo, hi = min(a, b), max(a, b)
            parent[hi] = lo

    inv, claim = set(), {}
    for m, t in props:
        q = int(st["mp_of"][t])
        if q >= 0:
            if q != m:
                union(m, q)
                inv |= {m, q}
        else:
            claim[t] = min(claim.get(t, m), m)
            inv.add(m)
    for m, t in props:
        if st["mp_of"][t] < 0 and claim[t] != m:
            union(m, claim[t])
    root = {m: find(m) for m in inv}
    surv = {}
    for m in inv:
        key = (len(_obs(st, m)), -m)
        r = root[m]
        surv[r] = max(surv.get(r, key), key)
    sv = {r: -v[1] for r, v in surv.items()}
    mp_of0 = st["mp_of"].copy()
    for s in range(R):
        groups = {}
        ent = []
        for kp in range(S):
            e = s * S + kp
            m = int(mp_of0[e])
            if m >= 0:
                if m not in inv:
                    continue
                g = root[m]
                key = 0 if m == sv[g] else ((1 << 28) | m)
                ent.append((kp, g, key, m))
            elif e in claim:
                g = root[claim[e]]
                ent.append((kp, g, (2 << 28) | kp, -1))
            else:
                continue
            groups[g] = min(groups.get(g, 1 << 62), ent[-1][2])
        for kp, g, key, mem in ent:
            e = s * S + kp
            win = groups[g] == key
            v = sv[g]
            if mem >= 0:
                if win:
                    if mem != v:
                        st["mp_of"][e] = v
                        st["okp"][mem][s] = -1
                        st["okp"][v][s] = kp
                else:
                    st["mp_of"][e] = -1
                    st["okp"][mem][s] = -1
            elif win:
                st["mp_of"][e] = v
                st["okp"][v][s] = kp
    for m in inv:
        if sv[root[m]] != m:
            st["rec"][m]["valid"] = 0


def camera_center(T):
    T = [F32(x) for x in T]
    px, py, pz = -T[4], -T[5], -T[6]
    qx, qy, qz, w = -T[0], -T[1], -T[2], T[3]
    u0, u1, u2 = qy * pz - qz * py, qz * px - qx * pz, qx * py - qy * px
    u0, u1, u2 = u0 + u0, u1 + u1, u2 + u2
    return ((px + w * u0) + (qy * u2 - qz * u1), (py + w * u1) + (qz * u0 - qx * u2),
            (pz + w * u2) + (qx * u1 - qy * u0))


def normal_depth(st, ring, m):
    """UpdateNormalAndDepth in float32, observations in slot order, the reference keyframe = the home slot."""
    S = st["S"]
    rec = st["rec"][m]
    P = [F32(x) for x in rec["pos"]]
    n0 = n1 = n2 = F32(0.0)
    n = 0
    with np.errstate(all="ignore"):
        for s, _ in _obs(st, m):
            ow = camera_center(st["tcw"][s])
            a = [P[i] - ow[i] for i in range(3)]
            nr = np.sqrt(a[0] * a[0] + (a[1] * a[1] + a[2] * a[2]))
            n0, n1, n2 = n0 + a[0] / nr, n1 + a[1] / nr, n2 + a[2] / nr
            n += 1
        if n == 0:
            return
        hs, hk = m // S, m % S
        ow = camera_center(st["tcw"][hs])
        c = [P[i] - ow[i] for i in range(3)]
        dist = np.sqrt(c[0] * c[0] + (c[1] * c[1] + c[2] * c[2]))
        sf = ring["sf"]
        level = min(max(int(ring["keys"][hs, hk]["octave"]), 0), len(sf) - 1)
        maxd = F32(dist * sf[level])
        rec["max_distance"] = maxd
        rec["min_distance"] = F32(maxd / sf[-1])
        fn = F32(n)
        rec["normal"] = (n0 / fn, n1 / fn, n2 / fn)


def _popc(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def distinctive(st, ring, m):
    obs = _obs(st, m)
    ds = [ring["desc"][s, k] for s, k in obs]
    N = len(ds)
    if N == 0:
        return
    D = np.zeros((N, N), np.int64)
    for i in range(N):
        for j in range(i + 1, N):
            D[i, j] = D[j, i] = _popc(ds[i], ds[j])
    best, bi = 1 << 30, 0
    for i in range(N):
        med = int(np.sort(D[i])[int(0.5 * (N - 1))])
        if med < best:
            best, bi = med, i
    st["rec"][m]["desc"] = ds[bi]


def refresh(st, ring, head, W):
    S = st["S"]
    touched = sorted({int(m) for m in st["mp_of"][head * S:(head + W) * S] if m >= 0})
    for m in touched:
        if st["rec"][m]["valid"]:
            normal_depth(st, ring, m)
            distinctive(st, ring, m)


def windows(st, ring, head, W, th, pcap, ecap):
    """LocalBundleAdjustment's windows: per new keyframe dict(slots, nloc, points (ids), edges (point, pose, slot, kp))
    or None when the window is not solved (no fixed keyframe / no MapPoint), 'overflow' past the caps."""
    S, R = st["S"], st["R"]
    out = []
    for w in range(W):
        j = head + w
        wt = np.zeros(R, np.int64)
        for m in st["mp_of"][j * S:(j + 1) * S]:
            if m >= 0:
                wt += st["okp"][m] >= 0
        wt[j] = 0
        cov = sorted([s for s in range(R) if wt[s] >= th], key=lambda s: (-wt[s], s))
        if not cov and wt.max() > 0:
            cov = [int(np.argmax(wt))]
        local = [j] + cov
        pts, seen = [], set()
        for s in local:
            for m in st["mp_of"][s * S:(s + 1) * S]:
                if m >= 0 and int(m) not in seen:
                    seen.add(int(m))
                    pts.append(int(m))
        if len(pts) > pcap:
            out.append("overflow")
            continue
        first = {}
        lset = set(local)
        for p, m in enumerate(pts):
            for s, _ in _obs(st, m):
                if s not in lset and s not in first:
                    first[s] = p
        fixed = sorted(first, key=lambda s: (first[s], s))
        if not fixed or not pts:
            out.append(None)
            continue
        slots = local + fixed
        pi = {s: i for i, s in enumerate(slots)}
        edges = []
        for p, m in enumerate(pts):
            for s, k in _obs(st, m):
                edges.append((p, pi[s], s, k))
        if len(edges) > ecap:
            out.append("overflow")
            continue
        out.append({"slots": slots, "nloc": len(local), "points": pts, "edges": edges})
    return out


def writeback(st, ring, wins, results):
    """Optimizer.cc:1413-1497 over the solved windows in order: results[w] = (pose_q, pose_t, point_xyz, chi2,
    depth_ok) (None for a skipped window)."""
    S = st["S"]
    erased = set()
    for w, (win, res) in enumerate(zip(wins, results)):
        if not isinstance(win, dict) or res is None:
            continue
        chi2, dok = res[3], res[4]
        for e, (p, _, s, _) in enumerate(win["edges"]):
            if chi2[e] > 5.991 or not dok[e]:
                m = win["points"][p]
                k = int(st["okp"][m][s])
                if k >= 0:
                    st["mp_of"][s * S + k] = -1
                    st["okp"][m][s] = -1
                    erased.add(m)
    newid = _repair(st, sorted(erased), lambda m, n: m in erased and n <= 2)

    def res_id(m):
        return newid.get(m, m)

    slot_last, lastw = {}, {}
    for w, (win, res) in enumerate(zip(wins, results)):
        if not isinstance(win, dict) or res is None:
            continue
        for i in range(win["nloc"]):
            slot_last[win["slots"][i]] = w
        for m in win["points"]:
            n = res_id(m)
            if n >= 0:
                lastw[n] = w
    for w, (win, res) in enumerate(zip(wins, results)):
        if not isinstance(win, dict) or res is None:
            continue
        q_all, t_all, x_all = res[0], res[1], res[2]
        for i in range(win["nloc"]):
            s = win["slots"][i]
            if slot_last[s] == w:
                q = [F32(v) for v in q_all[i]]
                nq = np.sqrt((q[0] * q[0] + q[2] * q[2]) + (q[1] * q[1] + q[3] * q[3]))
                st["tcw"][s, :4] = [x / nq for x in q]
                st["tcw"][s, 4:] = [F32(v) for v in t_all[i]]
        for p, m in enumerate(win["points"]):
            n = res_id(m)
            if n >= 0 and lastw[n] == w:
                st["rec"][n]["pos"] = [F32(v) for v in x_all[p]]
    for n in sorted(lastw):
        if st["rec"][n]["valid"]:
            normal_depth(st, ring, n)
    return newid, slot_last, lastw
