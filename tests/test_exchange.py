"""Shared-map update exchange (include/mam_exchange.h): the compact blocks the bench's LocalMapping
leg sends (CompactExchange: mam_exchange_pack_sources / mam_exchange_apply_compact).

CPU: the restatement (oracle/exchange_oracle.py) — the deduplicated block leaves exactly the tables the per-window
write-backs applied in order leave (the reference's sequential semantics), with the quaternion renormalised as
Sophus does; and the collective itself — CompactExchange.gather() at world_size 2 over gloo with windows that
overlap ACROSS ranks: both ranks receive identical bytes in rank order and end with the tables of rank 0's windows
then rank 1's applied in sequence. GPU: the pack / apply kernels byte-exact vs the restatement.
"""
import os
import socket

import numpy as np
import pytest

from oracle import exchange_oracle as xo


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _norm_orders_differ(q):
    """Sophus's (x^2 + z^2) + (y^2 + w^2) and the sequential ((x^2 + y^2) + z^2) + w^2 give different floats."""
    q = np.asarray(q, np.float32)
    sq = (q * q).astype(np.float32)
    n_seq = np.sqrt(np.float32(np.float32(np.float32(sq[0] + sq[1]) + sq[2]) + sq[3]))
    return not np.array_equal(xo.sophus_normalize(q), (q / n_seq).astype(np.float32))


def test_sophus_normalize_order():
    """KeyFrame::SetPose(SE3f(q.cast<float>(), t)) renormalises with Eigen's SSE reduction order; the order matters
    for ~15 % of quaternions (1 ulp), so the byte-exact tests below hold poses where the two orders differ."""
    q = np.array([0.0021944, 0.9986104, -0.0317063, 0.0418517], np.float32)
    rng = np.random.default_rng(1)
    found = [x for x in rng.normal(size=(400, 4)).astype(np.float32) if _norm_orders_differ(x)]
    assert len(found) > 20
    x, y, z, w = (np.float32(v) for v in found[0])
    n = np.sqrt(np.float32((x * x + z * z) + (y * y + w * w)))
    assert np.array_equal(xo.sophus_normalize(found[0]), (found[0] / n).astype(np.float32))
    assert np.abs(np.linalg.norm(xo.sophus_normalize(q).astype(np.float64)) - 1.0) < 1e-6


def test_world_windows_are_consistent():
    """The synthetic shared map (mam3slam_amd/world.py): windows cut from it are the reference's LBA graphs —
    50 local keyframes optimised (the init keyframe fixed), the keyframes observing their points outside the window
    fixed, every observation of a window point an edge — and overlapping windows share keyframes and MapPoints."""
    from mam3slam_amd import world as W

    wd = W.make_world(n_kf=200, seed=3)
    p0, k0, m0 = W.window(wd, 0)
    p1, k1, m1 = W.window(wd, 25)
    for p, k, s in ((p0, k0, 0), (p1, k1, 25)):
        assert np.all(np.diff(p.pose_id) > 0) and np.all(np.diff(p.point_id) > 0)
        local = (k >= s) & (k < s + 50) & (k != 0)
        assert np.array_equal(p.pose_fixed == 0, local)
        assert set(np.unique(p.edge_pose)) == set(range(len(k)))
        assert len(p.point_id) > 2500 and len(p.edge_point) > 8 * 2500 * 0.9
    assert len(np.intersect1d(k0, k1)) >= 25 and len(np.intersect1d(m0, m1)) > 1000
    assert p0.pose_fixed[0] == 1   # keyframe 0: the map's init keyframe (Optimizer.cc:1220)


def _windows_results(n_windows=4, seed=0):
    """Per-window LBA results over overlapping vertex sets (windows of one agent in one step)."""
    rng = np.random.default_rng(seed)
    res, wins = [], []
    for w in range(n_windows):
        pid = np.arange(10 * w, 10 * w + 25, dtype=np.int64)
        fixed = ((pid % 7) == 0).astype(np.uint8)
        mid = np.sort(rng.choice(np.arange(100 * w, 100 * w + 400), size=250, replace=False)).astype(np.int64) + 1000
        q = rng.normal(size=(len(pid), 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        t = rng.normal(size=(len(pid), 3))
        xyz = rng.normal(size=(len(mid), 3)) * 4
        bad = (rng.random(len(mid)) < 0.05).astype(np.uint8)
        res.append((q, t, pid, xyz, mid, bad))
        wins.append((pid, fixed, mid))
    return res, wins


def _sequential(res, wins, mp_base, kf_rows=64, mp_rows=1000, kf0=None, mp0=None):
    kf = np.zeros((kf_rows, 8), np.float32) if kf0 is None else kf0.copy()
    mp = np.zeros((mp_rows, 4), np.float32) if mp0 is None else mp0.copy()
    for (q, t, pid, xyz, mid, bad), (_, fixed, _) in zip(res, wins):
        xo.writeback(kf, mp, q, t, pid, fixed, xyz, np.asarray(mid) - mp_base, bad)
    return kf, mp


def test_compact_block_equals_sequential_writeback():
    """The deduplicated block (every vertex once, from the last window holding it) leaves the tables exactly as the
    windows' write-backs (Optimizer.cc:1478-1494) applied one after another do, at 16 / 32 bytes per record."""
    from mam3slam_amd.exchange import compact_block_bytes, dedup_sources

    res, wins = _windows_results()
    assert any(_norm_orders_differ(q) for r in res for q in r[0])
    mp_base = 1000
    kf_src, mp_src = dedup_sources(wins)
    ids_kf = [int(wins[w][0][i]) for w, i in kf_src]
    ids_mp = [int(wins[w][2][i]) for w, i in mp_src]
    assert ids_kf == sorted(set(ids_kf)) and ids_mp == sorted(set(ids_mp))
    blk = xo.pack_sources(res, kf_src, mp_src, mp_base, 0, len(kf_src), len(mp_src))
    assert len(blk) == compact_block_bytes(len(kf_src), len(mp_src))
    kf_a, mp_a = np.zeros((64, 8), np.float32), np.zeros((1000, 4), np.float32)
    assert xo.apply_compact(blk, 1, len(kf_src), len(mp_src), kf_a, mp_a) == 0
    kf_b, mp_b = _sequential(res, wins, mp_base)
    assert np.array_equal(kf_a, kf_b) and np.array_equal(mp_a, mp_b)
    per_window = sum(16 + 64 * (int((f == 0).sum()) + len(m)) for _, f, m in wins)   # round 2's 64-byte records
    assert len(blk) < per_window / 3
    # capacity overflow is flagged and the block is rejected whole
    small = xo.pack_sources(res, kf_src, mp_src, mp_base, 0, len(kf_src), len(mp_src) - 1)
    kf_c, mp_c = np.zeros((64, 8), np.float32), np.zeros((1000, 4), np.float32)
    assert xo.apply_compact(small, 1, len(kf_src), len(mp_src) - 1, kf_c, mp_c) == xo.ERR_ARG and not mp_c.any()


def _rank_windows(rank):
    """Rank r's windows of one step: 3 windows whose keyframes and MapPoints overlap each other AND the other rank's
    (keyframe ids 8 r + 10 w .., MapPoint ids from a pool shared by both ranks), as neighbouring agents' windows over
    a merged map do."""
    rng = np.random.default_rng(100 + rank)
    res, wins = [], []
    for w in range(3):
        pid = np.arange(8 * rank + 10 * w, 8 * rank + 10 * w + 20, dtype=np.int64)
        fixed = ((pid % 5) == 0).astype(np.uint8)
        mid = np.sort(rng.choice(np.arange(60 * w + 40 * rank, 60 * w + 40 * rank + 300), size=200,
                                 replace=False)).astype(np.int64) + 1000
        q = rng.normal(size=(len(pid), 4))
        q /= np.linalg.norm(q, axis=1, keepdims=True)
        res.append((q, rng.normal(size=(len(pid), 3)), pid, rng.normal(size=(len(mid), 3)) * 4, mid,
                    (rng.random(len(mid)) < 0.05).astype(np.uint8)))
        wins.append((pid, fixed, mid))
    return res, wins


def _compact_rank_main(rank, world, port, caps, outdir):
    import torch.distributed as dist

    from mam3slam_amd.exchange import CompactExchange, dedup_sources

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = CompactExchange(caps[0], caps[1], device="cpu")
    res, wins = _rank_windows(rank)
    kf_src, mp_src = dedup_sources(wins)
    blk = xo.pack_sources(res, kf_src, mp_src, 1000, ex.rank, caps[0], caps[1])
    ex.send.numpy()[:] = np.frombuffer(blk, np.uint8)
    got = ex.gather().numpy().copy()
    kf = np.zeros((64, 8), np.float32)
    mp = np.zeros((1000, 4), np.float32)
    st = xo.apply_compact(got.tobytes(), world, caps[0], caps[1], kf, mp)
    np.savez(os.path.join(outdir, f"c{rank}.npz"), got=got, kf=kf, mp=mp, st=st)
    dist.destroy_process_group()


def test_compact_gather_gloo_world2(tmp_path):
    """The all-gather the bench's exchange takes (CompactExchange.gather, world 2, gloo), with windows overlapping
    across the ranks: identical bytes on both ranks in rank order, and the applied tables equal rank 0's windows then
    rank 1's written back in sequence (the higher rank wins a conflict)."""
    import torch.multiprocessing as mp

    from mam3slam_amd.exchange import compact_block_bytes, dedup_sources

    world = 2
    srcs = [dedup_sources(_rank_windows(r)[1]) for r in range(world)]
    caps = (max(len(k) for k, _ in srcs) + 4, max(len(m) for _, m in srcs) + 4)   # the all-reduce MAX of the bench
    mp.start_processes(_compact_rank_main, args=(world, _free_port(), caps, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r0, r1 = (np.load(tmp_path / f"c{r}.npz") for r in range(world))
    assert int(r0["st"]) == 0 == int(r1["st"])
    assert np.array_equal(r0["got"], r1["got"])
    assert np.array_equal(r0["kf"], r1["kf"]) and np.array_equal(r0["mp"], r1["mp"])
    bb = compact_block_bytes(*caps)
    for r in range(world):
        res, wins = _rank_windows(r)
        exp = xo.pack_sources(res, *srcs[r], 1000, r, *caps)
        assert r0["got"][r * bb:(r + 1) * bb].tobytes() == exp, f"block {r} not in rank order"
    k0 = set(int(x) for _, _, pid, _, _, _ in _rank_windows(0)[0] for x in pid)
    k1 = set(int(x) for _, _, pid, _, _, _ in _rank_windows(1)[0] for x in pid)
    assert len(k0 & k1) > 10   # the ranks' windows really conflict
    res0, wins0 = _rank_windows(0)
    res1, wins1 = _rank_windows(1)
    kf_s, mp_s = _sequential(res0 + res1, wins0 + wins1, 1000)
    assert np.array_equal(r0["kf"], kf_s) and np.array_equal(r0["mp"], mp_s)


@pytest.mark.gpu
def test_compact_pack_apply_kernels(gpu_lib):
    """mam_exchange_pack_sources / mam_exchange_apply_compact byte-exact vs the restatement (including quaternions
    whose Sophus renormalisation differs from the sequential sum order), two agents' blocks applied in agent order,
    and the applied tables equal the agents' windows written back in sequence."""
    import torch

    from mam3slam_amd.exchange import CompactExchange, MapWindow, compact_block_bytes, dedup_sources

    dev = torch.device("cuda")
    mp_base = 1000
    blocks, keep = [], []
    data = [_windows_results(seed=agent) for agent in range(2)]
    srcs = [dedup_sources(wins) for _, wins in data]
    caps = (max(len(k) for k, _ in srcs) + 8, max(len(m) for _, m in srcs) + 8)   # the same block on every agent
    for agent in range(2):
        res, wins = data[agent]
        kf_src, mp_src = srcs[agent]
        ex = CompactExchange(caps[0], caps[1], device=dev)
        ex.rank = agent
        desc = (MapWindow * len(res))()
        for w, (q, t, pid, xyz, mid, bad) in enumerate(res):
            T = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (q, t, pid, wins[w][1], xyz, mid, bad)]
            keep += T
            d = desc[w]
            d.n_poses, d.n_points = len(pid), len(mid)
            d.pose_q, d.pose_t, d.pose_id, d.pose_fixed = T[0].data_ptr(), T[1].data_ptr(), T[2].data_ptr(), T[3].data_ptr()
            d.point_xyz, d.point_id, d.point_bad = T[4].data_ptr(), T[5].data_ptr(), T[6].data_ptr()
        d_desc = torch.from_numpy(np.frombuffer(bytes(desc), np.uint8).copy()).to(dev)
        d_k, d_m = torch.from_numpy(kf_src).to(dev), torch.from_numpy(mp_src).to(dev)
        keep += [d_desc, d_k, d_m]
        ex.send.fill_(0xCD)
        ex.pack(d_desc.data_ptr(), len(res), d_k.data_ptr(), len(kf_src), d_m.data_ptr(), len(mp_src), mp_base)
        torch.cuda.synchronize()
        exp = xo.pack_sources(res, kf_src, mp_src, mp_base, agent, caps[0], caps[1])
        got = ex.send.cpu().numpy().tobytes()
        nk, nm = len(kf_src), len(mp_src)
        used = [(0, 16), (16, 16 + 32 * nk), (16 + 32 * caps[0], 16 + 32 * caps[0] + 16 * nm)]
        for a, b in used:
            assert got[a:b] == exp[a:b], (agent, a, b)
        blocks.append(exp)
    assert compact_block_bytes(*caps) == len(blocks[0])
    gathered = b"".join(blocks)
    ex.recv = torch.from_numpy(np.frombuffer(gathered, np.uint8).copy()).to(dev)
    ex.world = 2
    kf = torch.zeros((128, 8), dtype=torch.float32, device=dev)
    mpt = torch.zeros((1000, 4), dtype=torch.float32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    ex.apply(kf.data_ptr(), 128, mpt.data_ptr(), 1000, status.data_ptr())
    torch.cuda.synchronize()
    kf_o, mp_o = np.zeros((128, 8), np.float32), np.zeros((1000, 4), np.float32)
    assert xo.apply_compact(gathered, 2, caps[0], caps[1], kf_o, mp_o) == 0 == int(status.item())
    assert np.array_equal(kf.cpu().numpy(), kf_o) and np.array_equal(mpt.cpu().numpy(), mp_o)
    assert any(_norm_orders_differ(q) for r in data[0][0] for q in r[0])
    kf_s, mp_s = _sequential(data[0][0] + data[1][0], data[0][1] + data[1][1], mp_base, 128, 1000)
    assert np.array_equal(kf.cpu().numpy(), kf_s) and np.array_equal(mpt.cpu().numpy(), mp_s)


@pytest.mark.gpu
def test_copy_rows_and_perturb_kernels(gpu_lib):
    """mam_copy_rows (the ring ingest's one launch) against torch row indexing, incl. an offset source table, a
    4-byte column of a strided table and the flags; mam_map_perturb: unit quaternions with w >= 0, only the listed
    rows changed, deterministic in the seed."""
    import torch

    from mam3slam_amd.exchange import copy_rows, map_perturb

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    A = torch.randint(0, 256, (10, 100), dtype=torch.uint8, generator=g).to(dev)
    B = torch.zeros((7, 100), dtype=torch.uint8, device=dev)
    cnt = torch.randint(0, 1000, (10, 2), dtype=torch.int32, generator=g).to(dev)
    col = torch.zeros(7, dtype=torch.int32, device=dev)
    F = torch.randint(0, 256, (20, 48), dtype=torch.uint8, generator=g).to(dev)
    G = torch.zeros((7, 48), dtype=torch.uint8, device=dev)
    o1 = torch.randint(-1, 3, (10, 30), dtype=torch.int32, generator=g).to(dev)
    o2 = torch.randint(-1, 3, (10, 30), dtype=torch.int32, generator=g).to(dev)
    fl = torch.zeros((7, 30), dtype=torch.uint8, device=dev)
    src, dst = [4, 0, 9], [6, 2, 3]
    copy_rows([(A.data_ptr(), B.data_ptr(), 100, 100, 100, 0), (cnt.data_ptr(), col.data_ptr(), 4, 8, 4, 0),
               (F.data_ptr(), G.data_ptr(), 48, 48, 48, 10)], src, dst,
              (o1.data_ptr(), o2.data_ptr(), 4 * 30, 30, fl.data_ptr(), 30))
    torch.cuda.synchronize()
    for s_, d_ in zip(src, dst):
        assert torch.equal(B[d_], A[s_]) and int(col[d_]) == int(cnt[s_, 0]) and torch.equal(G[d_], F[10 + s_])
        assert torch.equal(fl[d_], ((o1[s_] >= 0) | (o2[s_] >= 0)).to(torch.uint8))
    for r in set(range(7)) - set(dst):
        assert int(B[r].sum()) == 0 and int(fl[r].sum()) == 0
    kf = torch.zeros((5, 8), dtype=torch.float32, device=dev)
    kf[:, 3] = 1.0
    mp = torch.zeros((9, 4), dtype=torch.float32, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    ki, mi = torch.tensor([1, 3], device=dev), torch.tensor([0, 5, 8], device=dev)
    outs = []
    for _ in range(2):
        k2, m2 = kf.clone(), mp.clone()
        map_perturb(k2.data_ptr(), 5, ki.data_ptr(), 2, m2.data_ptr(), 9, mi.data_ptr(), 3, 1234, 0.004, 0.012, 0.017,
                    st.data_ptr())
        torch.cuda.synchronize()
        outs.append((k2, m2))
    assert int(st) == 0
    k2, m2 = outs[0]
    assert torch.equal(k2, outs[1][0]) and torch.equal(m2, outs[1][1])
    q = k2[ki, :4]
    assert torch.allclose(q.norm(dim=1), torch.ones(2, device=dev), atol=1e-6) and bool((q[:, 3] >= 0).all())
    assert bool((k2[[0, 2, 4]] == kf[[0, 2, 4]]).all()) and bool((m2[[1, 2, 3, 4, 6, 7]] == 0).all())
    assert float(m2[mi, :3].abs().max()) > 0 and float(m2[mi, :3].abs().max()) < 0.2
