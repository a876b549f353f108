"""Shared-map update exchange (include/mam_exchange.h).

CPU: the collective itself — MapUpdateExchange.gather() at world_size 2 over gloo — with blocks packed and applied
by the numpy restatement (oracle/exchange_oracle.py): both ranks receive identical bytes in rank order and end with
identical tables where the higher agent wins a conflict. GPU: the pack / apply kernels byte-exact vs the
restatement, including conflicts, bad flags, out-of-range ids and capacity overflow.
"""
import os
import socket

import numpy as np
import pytest

from mam3slam_amd.exchange import MapUpdateExchange
from oracle import exchange_oracle as xo


def _agent_update(agent, n_poses=12, n_points=300, shared=200, seed=0):
    """An agent's LBA write-back: poses ids 10*agent.., points drawn from a shared id pool (merged map)."""
    rng = np.random.default_rng(seed + 17 * agent)
    q = rng.normal(size=(n_poses, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    t = rng.normal(size=(n_poses, 3))
    pid = np.arange(n_poses, dtype=np.int64) + 5 * agent          # overlapping keyframe ids
    fixed = (rng.random(n_poses) < 0.3).astype(np.uint8)
    mid = np.sort(rng.choice(shared + n_points, size=n_points, replace=False)).astype(np.int64)
    xyz = rng.normal(size=(n_points, 3)) * 3
    bad = (rng.random(n_points) < 0.05).astype(np.uint8)
    return q, t, pid, fixed, xyz, mid, bad


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, cap, outdir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = MapUpdateExchange(capacity=cap, device="cpu")
    q, t, pid, fixed, xyz, mid, bad = _agent_update(rank)
    blk = xo.pack_lba(q, t, pid, fixed, xyz, mid, bad, rank, cap)
    ex.send.numpy()[:] = blk.view(np.uint8)
    got = ex.gather().numpy().copy()
    kf = np.zeros((64, 8), np.float32)
    mp = np.zeros((1024, 4), np.float32)
    st = xo.apply(got.view(xo.UPDATE_DTYPE), world, cap, kf, mp)
    np.savez(os.path.join(outdir, f"r{rank}.npz"), got=got, kf=kf, mp=mp, st=st)
    dist.destroy_process_group()


def test_gather_gloo_world2(tmp_path):
    import torch.multiprocessing as mp

    cap, world = 512, 2
    mp.start_processes(_rank_main, args=(world, _free_port(), cap, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r0, r1 = (np.load(tmp_path / f"r{r}.npz") for r in range(world))
    assert np.array_equal(r0["got"], r1["got"])
    assert np.array_equal(r0["kf"], r1["kf"]) and np.array_equal(r0["mp"], r1["mp"])
    assert int(r0["st"]) == 0
    blocks = r0["got"].view(xo.UPDATE_DTYPE).reshape(world, cap + 1)
    for a in range(world):
        exp = xo.pack_lba(*_agent_update(a), a, cap)
        assert np.array_equal(blocks[a].view(np.uint8), exp.view(np.uint8)), f"block {a} not in rank order"
    # conflicts: ids written by both agents hold agent 1's values (applied last)
    q1, t1, pid1, fx1, xyz1, mid1, bad1 = _agent_update(1)
    for i, m in enumerate(mid1):
        assert np.array_equal(r0["mp"][m, :3], xyz1[i].astype(np.float32))
    b1 = xo.pack_lba(q1, t1, pid1, fx1, xyz1, mid1, bad1, 1, cap)
    for u in b1[1:1 + int(b1[0]["id"])]:
        if u["kind"] == xo.UPDATE_KF:
            assert np.array_equal(r0["kf"][u["id"], :7], u["v"]) and r0["kf"][u["id"], 7] == 1.0


def test_pack_capacity_and_header():
    q, t, pid, fixed, xyz, mid, bad = _agent_update(0)
    n_opt = int((fixed == 0).sum())
    blk = xo.pack_lba(q, t, pid, fixed, xyz, mid, bad, 3, n_opt + len(mid))
    assert blk[0]["id"] == n_opt + len(mid) and blk[0]["agent"] == 3
    assert (blk["kind"][1:1 + n_opt] == xo.UPDATE_KF).all() and (blk["kind"][1 + n_opt:] == xo.UPDATE_MP).all()
    small = xo.pack_lba(q, t, pid, fixed, xyz, mid, bad, 3, n_opt + len(mid) - 1)
    assert small[0]["id"] == xo.ERR_CAPACITY
    kf, mpt = np.zeros((64, 8), np.float32), np.zeros((1024, 4), np.float32)
    assert xo.apply(small, 1, n_opt + len(mid) - 1, kf, mpt) == xo.ERR_ARG and not kf.any()


@pytest.mark.gpu
def test_pack_apply_kernels(gpu_lib):
    import torch

    dev = torch.device("cuda")
    cap, agents = 600, 3
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    ex = MapUpdateExchange(capacity=cap, device=dev)
    blocks = []
    for a in range(agents):
        q, t, pid, fixed, xyz, mid, bad = _agent_update(a, seed=5)
        T = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (q, t, pid, fixed, xyz, mid, bad)]
        ex.send.fill_(0xAB)
        torch.cuda.synchronize()
        ex.pack_lba(T[0].data_ptr(), T[1].data_ptr(), T[2].data_ptr(), T[3].data_ptr(), len(pid), T[4].data_ptr(),
                    T[5].data_ptr(), T[6].data_ptr(), len(mid), stream=st.cuda_stream, agent=a)
        torch.cuda.synchronize()
        got = ex.send.cpu().numpy().view(xo.UPDATE_DTYPE)
        exp = xo.pack_lba(q, t, pid, fixed, xyz, mid, bad, a, cap)
        n = int(exp[0]["id"])
        assert np.array_equal(got[:1 + n].view(np.uint8), exp[:1 + n].view(np.uint8)), f"agent {a} pack"
        blocks.append(exp)
    # an out-of-range id in agent 2's block -> status ERR_ARG, the record skipped
    blocks[2][5]["id"] = 10 ** 6
    gathered = np.concatenate(blocks)
    d_g = torch.from_numpy(gathered.view(np.uint8).copy()).to(dev)
    kf = torch.zeros((64, 8), dtype=torch.float32, device=dev)
    mpt = torch.zeros((1024, 4), dtype=torch.float32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    ex.apply(kf.data_ptr(), 64, mpt.data_ptr(), 1024, status.data_ptr(), stream=st.cuda_stream,
             gathered=d_g.data_ptr(), n_agents=agents)
    torch.cuda.synchronize()
    kf_o, mp_o = np.zeros((64, 8), np.float32), np.zeros((1024, 4), np.float32)
    st_o = xo.apply(gathered, agents, cap, kf_o, mp_o)
    assert int(status.item()) == st_o == xo.ERR_ARG
    assert np.array_equal(kf.cpu().numpy(), kf_o) and np.array_equal(mpt.cpu().numpy(), mp_o)
    # capacity overflow is reported in the header
    q, t, pid, fixed, xyz, mid, bad = _agent_update(0, n_points=cap)
    T = [torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (q, t, pid, fixed, xyz, mid, bad)]
    ex.pack_lba(T[0].data_ptr(), T[1].data_ptr(), T[2].data_ptr(), T[3].data_ptr(), len(pid), T[4].data_ptr(),
                T[5].data_ptr(), T[6].data_ptr(), len(mid), stream=st.cuda_stream, agent=0)
    torch.cuda.synchronize()
    assert int(ex.send.cpu().numpy().view(xo.UPDATE_DTYPE)[0]["id"]) == xo.ERR_CAPACITY


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


def test_compact_block_equals_per_window_blocks():
    """The deduplicated block (every vertex once, from the last window holding it) leaves the tables exactly as the
    per-window write-backs applied in window order do, at 16 / 32 bytes per record instead of 64."""
    from mam3slam_amd.exchange import compact_block_bytes, dedup_sources

    res, wins = _windows_results()
    mp_base = 1000
    kf_src, mp_src = dedup_sources(wins)
    ids_kf = [int(wins[w][0][i]) for w, i in kf_src]
    ids_mp = [int(wins[w][2][i]) for w, i in mp_src]
    assert ids_kf == sorted(set(ids_kf)) and ids_mp == sorted(set(ids_mp))
    blk = xo.pack_sources(res, kf_src, mp_src, mp_base, 0, len(kf_src), len(mp_src))
    assert len(blk) == compact_block_bytes(len(kf_src), len(mp_src))
    kf_a, mp_a = np.zeros((64, 8), np.float32), np.zeros((1000, 4), np.float32)
    assert xo.apply_compact(blk, 1, len(kf_src), len(mp_src), kf_a, mp_a) == 0
    kf_b, mp_b = np.zeros((64, 8), np.float32), np.zeros((1000, 4), np.float32)
    cap = max(int((f == 0).sum()) + len(m) for _, f, m in wins)
    blocks = [xo.pack_lba(q, t, pid, wins[w][1], xyz, mid - mp_base, bad, 0, cap)
              for w, (q, t, pid, xyz, mid, bad) in enumerate(res)]
    assert xo.apply(np.concatenate(blocks), len(blocks), cap, kf_b, mp_b) == 0
    assert np.array_equal(kf_a, kf_b) and np.array_equal(mp_a, mp_b)
    assert len(blk) < sum(b.nbytes for b in blocks) / 3
    # capacity overflow is flagged and the block is rejected whole
    small = xo.pack_sources(res, kf_src, mp_src, mp_base, 0, len(kf_src), len(mp_src) - 1)
    kf_c, mp_c = np.zeros((64, 8), np.float32), np.zeros((1000, 4), np.float32)
    assert xo.apply_compact(small, 1, len(kf_src), len(mp_src) - 1, kf_c, mp_c) == xo.ERR_ARG and not mp_c.any()


@pytest.mark.gpu
def test_compact_pack_apply_kernels(gpu_lib):
    """mam_exchange_pack_sources / mam_exchange_apply_compact byte-exact vs the restatement, two agents' blocks
    applied in agent order."""
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
