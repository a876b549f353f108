"""GPU: the device map LocalMapping works on (include/mam_ringmap.h) — MapPoint identities shared across the keyframe
ring, LocalMapping's edits and LocalBundleAdjustment's window / write-back over them — every phase of a LocalMapping
run compared with the host restatement (tests/ringmap_host.py) applied to the device state before the phase:
eviction + culling, CreateNewMapPoints, Fuse's Replace / AddObservation, the descriptor / normal / depth refresh
(byte-exact map state), the windows by the reference's rule (Optimizer.cc:1118-1186: union of the local keyframes'
MapPoints, fixed = their other observers; every array byte-exact), the solve against the oracle (identical Levenberg
control flow, 1e-4) and the write-back (Optimizer.cc:1413-1497: outlier erase, SetPose, SetWorldPos,
UpdateNormalAndDepth; byte-exact)."""
import numpy as np
import pytest

import ringmap_host as H

pytestmark = pytest.mark.gpu

PATH = (16.0, 0.25, 4096)


def _setup(cfg="c1", B=64, runs=6):
    import torch

    import bench
    from mam3slam_amd.mapping import NewMapPointsLeg, RingMappingLeg

    dev = torch.device("cuda", 0)
    conf = dict(bench.CONFIGS[cfg], path=PATH)
    tr = bench.TrackingLeg(conf, B, 1, 0, dev)
    nm = NewMapPointsLeg(tr, B // 8, dev)
    leg = RingMappingLeg(nm, 0, 1, dev, pcap=8192, ecap=131072)
    for r in range(runs):
        tr.step()
        leg.run(r, nm.ingest(r))
    torch.cuda.synchronize()
    tr.step()
    return tr, nm, leg, nm.ingest(runs)


def _ring(nm, tr):
    from mam3slam_amd.match import FUSE_MP_DTYPE
    from mam3slam_amd.orb import KP_DTYPE

    R, S = nm.R, nm.S
    sf = np.asarray(tr.F0.scale_factors, np.float32)
    return {"keys": nm.keys.cpu().numpy().view(KP_DTYPE).reshape(R, S), "desc": nm.desc.cpu().numpy(),
            "cnt": nm.cnt.cpu().numpy()[:, 0].copy(), "kp_rec": nm.fmp.cpu().numpy().view(FUSE_MP_DTYPE).reshape(-1),
            "sf": sf, "inv_s2": (np.float32(1.0) / np.asarray(tr.F0.level_sigma2, np.float32)).astype(np.float32)}


def _state(nm):
    s = nm.map.snapshot()
    s.update(R=nm.R, S=nm.S)
    return s


def _same(dev, host, what):
    assert np.array_equal(dev["mp_of"], host["mp_of"]), f"{what}: mp_of"
    assert np.array_equal(dev["okp"], host["okp"]), f"{what}: okp"
    live = dev["rec"]["valid"] != 0
    assert np.array_equal(live, host["rec"]["valid"] != 0), f"{what}: live MapPoints"
    assert np.array_equal(dev["rec"][live].view(np.uint8), host["rec"][live].view(np.uint8)), f"{what}: records"
    assert np.array_equal(dev["born"][live], host["born"][live]), f"{what}: born"
    assert np.array_equal(dev["tcw"].view(np.uint32), host["tcw"].view(np.uint32)), f"{what}: poses"


def test_ringmap_run_matches_host_restatement(gpu_lib, oracle):
    import torch

    tr, nm, leg, item = _setup()
    snaps = {}

    def hook(phase):
        torch.cuda.synchronize()
        snaps[phase] = _state(nm)
        if phase in ("search", "fuse_search"):
            snaps[phase + "_out"] = (nm.out.cpu().numpy().copy(), nm.fwd_idx.cpu().numpy().copy(),
                                     nm.bwd_idx.cpu().numpy().copy(), nm.pairs_d.cpu().numpy().copy())

    st = leg.stream
    nm.process(st, item, hook=hook)
    torch.cuda.synchronize()
    ring = _ring(nm, tr)
    head, W, run = nm.head, nm.W, nm.run_index
    # eviction + MapPointCulling
    h = {k: (v.copy() if hasattr(v, "copy") else v) for k, v in snaps["insert"].items()}
    H.evict(h, head, W, run)
    _same(snaps["evict"], h, "evict")
    assert np.array_equal(nm.has_mp.cpu().numpy().reshape(-1) != 0, snaps["evict"]["mp_of"] >= 0)
    # CreateNewMapPoints from the device's triangulation matches
    out, _, _, pairs = snaps["search_out"]
    h = {k: (v.copy() if hasattr(v, "copy") else v) for k, v in snaps["search"].items()}
    H.create(h, ring, head, W, pairs, nm.NN, out, run)
    _same(snaps["create"], h, "create")
    n_new = int(((snaps["create"]["mp_of"] >= 0).reshape(nm.R, nm.S)[head:head + W]).sum())
    assert n_new > 50 * W, n_new
    # the Fuse lists the searches read
    lists = nm.map.lists.cpu().numpy().view(h["rec"].dtype).reshape(-1)
    hl = H.gather(h)
    assert np.array_equal(lists["valid"], hl["valid"]) and np.array_equal(lists[hl["valid"] != 0].view(np.uint8),
                                                                          hl[hl["valid"] != 0].view(np.uint8))
    # the Fuse side effects from the device's Fuse matches
    _, fwd, bwd, _ = snaps["fuse_search_out"]
    h = {k: (v.copy() if hasattr(v, "copy") else v) for k, v in snaps["fuse_search"].items()}
    H.fuse_apply(h, ring, head, W, pairs, nm.NN, nm.NB, fwd, bwd)
    import os

    if os.environ.get("MAM_RINGMAP_DUMP"):   # the inputs and both results of the phase, for a host diagnosis
        pre, post = snaps["fuse_search"], snaps["fuse_apply"]
        np.savez_compressed(os.environ["MAM_RINGMAP_DUMP"], head=head, W=W, NN=nm.NN, NB=nm.NB, pairs=pairs, fwd=fwd,
                            bwd=bwd, cnt=ring["cnt"], **{"pre_" + k: v for k, v in pre.items() if k not in ("R", "S")},
                            **{"dev_" + k: v for k, v in post.items() if k not in ("R", "S")}, R=nm.R, S=nm.S)
    _same(snaps["fuse_apply"], h, "fuse_apply")
    merged = int((snaps["fuse_search"]["rec"]["valid"] != 0).sum() - (snaps["fuse_apply"]["rec"]["valid"] != 0).sum())
    assert merged > 0, "no Replace merge exercised"
    # ComputeDistinctiveDescriptors + UpdateNormalAndDepth
    H.refresh(h, ring, head, W)
    _same(snaps["refresh"], h, "refresh")
    # the windows
    rl = leg.rl
    rl.assemble(st)
    torch.cuda.synchronize()
    hw = H.windows(h, ring, head, W, rl.COVIS_TH, rl.pcap, rl.ecap)
    counts = rl.counts.cpu().numpy()
    pslot, pid = rl.pose_slot.cpu().numpy(), rl.point_id.cpu().numpy()
    solved = 0
    for w in range(W):
        if hw[w] is None:
            assert tuple(counts[w]) == (0, 0, 0, 0)
            continue
        win = hw[w]
        np_, L, E = len(win["slots"]), len(win["points"]), len(win["edges"])
        assert tuple(counts[w]) == (np_, L, E, win["nloc"]), (w, counts[w], (np_, L, E, win["nloc"]))
        assert np.array_equal(pslot[w, :np_], win["slots"]) and np.array_equal(pid[w, :L], win["points"])
        b = {k: v.cpu().numpy() for k, v in rl.bufs[w].items()}
        assert np.array_equal(b["pose_q"][:np_], h["tcw"][win["slots"], :4].astype(np.float64))
        assert np.array_equal(b["pose_t"][:np_], h["tcw"][win["slots"], 4:].astype(np.float64))
        assert np.array_equal(b["pose_fixed"][:np_], (np.arange(np_) >= win["nloc"]).astype(np.uint8))
        assert np.array_equal(b["point_xyz"][:L], h["rec"][win["points"]]["pos"].astype(np.float64))
        ed = np.array(win["edges"]).reshape(-1, 4)
        assert np.array_equal(b["edge_point"][:E], ed[:, 0]) and np.array_equal(b["edge_pose"][:E], ed[:, 1])
        kp = ring["keys"][ed[:, 2], ed[:, 3]]
        assert np.array_equal(b["edge_obs"][:E], np.stack([kp["x"], kp["y"]], 1).astype(np.float64))
        assert np.array_equal(b["edge_inv_sigma2"][:E], ring["inv_s2"][kp["octave"]].astype(np.float64))
        solved += 1
    assert solved > 0, "no window with fixed keyframes"
    # the solve against the oracle
    stats = rl.solve(st)
    for w in rl.valid[:2]:
        prob = rl.window(w)
        q, t, x, its, trials, stt, ic, fc = rl.result(w)
        ro = oracle.lba_solve(prob)
        assert stt == 0 and (its, trials) == (ro.iterations, ro.lm_trials), (w, its, trials, ro.iterations, ro.lm_trials)
        rel = np.abs(x - ro.point_xyz).max() / np.abs(ro.point_xyz).max()
        assert rel <= 1e-4 and np.abs(t - ro.pose_t).max() <= 1e-4 * max(np.abs(ro.pose_t).max(), 1.0)
    # the write-back
    torch.cuda.synchronize()
    before = _state(nm)
    results = []
    for w in range(W):
        if w not in rl.valid:
            results.append(None)
            continue
        P, L, E = rl._size(w)
        b = rl.bufs[w]
        results.append((b["out_q"].cpu().numpy()[:P], b["out_t"].cpu().numpy()[:P], b["out_xyz"].cpu().numpy()[:L],
                        b["out_chi2"].cpu().numpy()[:E], b["out_depth"].cpu().numpy()[:E]))
    rl.writeback(st)
    torch.cuda.synchronize()
    after = _state(nm)
    h = {k: (v.copy() if hasattr(v, "copy") else v) for k, v in before.items()}
    H.writeback(h, ring, [hw[w] if w in rl.valid else None for w in range(W)], results)
    _same(after, h, "writeback")
    assert any(s[1] > 0 for s in stats)
