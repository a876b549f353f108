"""GPU parity: the HIP ORB extractor (through the C-ABI) vs the CPU oracle, bit-exact.

Stages are compared separately (pyramid, blurred levels, per-level FAST candidates) so a failure points at
one kernel; the end-to-end check compares every keypoint field and every descriptor byte, in output order,
plus the returned monoIndex (reference semantics: src/ORBextractor.cc:1086-1168).
"""
import numpy as np
import pytest

from mam3slam_amd import synth

pytestmark = pytest.mark.gpu

# (w, h, nfeatures) — BASELINE.json configs (640x480/1000, 1280x720/2000), the testMultiAgentSystem YAML
# (960x960, 700 features, test/settingsForTest_00.yaml:37) and the 5x init extractor (Tracking.cc:606).
CASES = [(640, 480, 1000), (1280, 720, 2000), (960, 960, 700), (640, 480, 5000)]


def _extractor(nfeat, fp_policy=0):
    from mam3slam_amd import ORBextractor

    return ORBextractor(nfeat, 1.2, 8, 20, 7, fp_policy=fp_policy)


def _first_diff(a, b):
    idx = np.nonzero(a != b)
    return tuple(int(i[0]) for i in idx) if len(idx[0]) else None


def _assert_kps_equal(kg, dg, mg, ko, do, mo, tag):
    assert len(kg) == len(ko), f"{tag}: n {len(kg)} vs oracle {len(ko)}"
    assert mg == mo, f"{tag}: monoIndex {mg} vs {mo}"
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        a, b = kg[f], ko[f]
        if f in ("x", "y", "size", "angle", "response"):
            a, b = a.view(np.uint32), b.view(np.uint32)   # bit-exact floats
        d = _first_diff(a, b)
        assert d is None, f"{tag}: field {f} differs first at {d}: gpu={kg[d[0]]} oracle={ko[d[0]]}"
    d = _first_diff(dg, do)
    assert d is None, f"{tag}: descriptor differs first at {d}: gpu={dg[d[0]]} oracle={do[d[0]]} kp={ko[d[0]]}"


@pytest.mark.parametrize("w,h,nfeat", CASES[:3])
def test_pyramid_blur_candidates(gpu_lib, oracle, w, h, nfeat):
    ext = _extractor(nfeat)
    img = synth.make_frame(w, h, agent=1, frame=3)
    ext(img)
    p = oracle.params(nfeat)
    levels = oracle.pyramid(img, p)
    for l, lev in enumerate(levels):
        g = ext.level(l)
        d = _first_diff(g, lev)
        assert d is None, f"level {l} pixel {d}: gpu={g[d]} oracle={lev[d]}"
        gb = ext.debug_blurred(l)
        ob = oracle.gaussian7(lev)
        d = _first_diff(gb, ob)
        assert d is None, f"blurred level {l} pixel {d}: gpu={gb[d]} oracle={ob[d]}"
        cand_o, _ = oracle.level_stage(img, l, p)
        cand_g = ext.debug_candidates(l)
        assert len(cand_g) == len(cand_o), f"level {l}: {len(cand_g)} candidates vs oracle {len(cand_o)}"
        d = _first_diff(cand_g, cand_o)
        assert d is None, f"level {l} candidate {d}: gpu={oracle.unpack(cand_g[d])} oracle={oracle.unpack(cand_o[d])}"


@pytest.mark.parametrize("w,h,nfeat", CASES)
def test_extract_bit_exact(gpu_lib, oracle, w, h, nfeat):
    ext = _extractor(nfeat)
    p = oracle.params(nfeat)
    for fr in range(2):
        img = synth.make_frame(w, h, agent=0, frame=fr)
        kg, dg, mg = ext(img)
        ko, do, mo = oracle.extract(img, p)
        _assert_kps_equal(kg, dg, mg, ko, do, mo, f"{w}x{h}/{nfeat} frame {fr}")


@pytest.mark.parametrize("policy", [1, 2, 4, 5])
def test_extract_fp_policies(gpu_lib, oracle, policy):
    """Non-default arithmetic policies (mam_orb.h MAM_FP_*: uncontracted GET_VALUE, glibc's SSE2 sincosf, correctly
    rounded trig) are bit-exact against the oracle under the same policy."""
    ext = _extractor(1000, fp_policy=policy)
    img = synth.make_frame(640, 480, agent=2, frame=5)
    kg, dg, mg = ext(img)
    ko, do, mo = oracle.extract(img, oracle.params(1000, fp_policy=policy))
    _assert_kps_equal(kg, dg, mg, ko, do, mo, f"fp_policy={policy}")


def test_lapping_area_placement(gpu_lib, oracle):
    ext = _extractor(1000)
    img = synth.make_frame(640, 480, agent=3, frame=1)
    for lap in [(0, 1000), (200, 400), (700, 900), (0, 0)]:
        kg, dg, mg = ext(img, None, lap)
        ko, do, mo = oracle.extract(img, oracle.params(1000), lap)
        _assert_kps_equal(kg, dg, mg, ko, do, mo, f"lap {lap}")


def test_batch_device_matches_single(gpu_lib, oracle):
    import torch

    from mam3slam_amd.orb import KP_DTYPE

    w, h, F = 640, 480, 6
    ext = _extractor(1000)
    imgs = np.stack([synth.make_frame(w, h, agent=4, frame=i) for i in range(F)])
    cap = ext.max_keypoints()
    d_img = torch.from_numpy(imgs).cuda()
    d_kps = torch.zeros((F, cap * 28), dtype=torch.uint8, device="cuda")
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros((F, 2), dtype=torch.int32, device="cuda")
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    ext.extract_batch_device(d_img.data_ptr(), F, w, h, w, w * h, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                             d_cnt.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    cnt = d_cnt.cpu().numpy()
    kps = d_kps.cpu().numpy().view(KP_DTYPE).reshape(F, cap)
    desc = d_desc.cpu().numpy()
    for i in range(F):
        ko, do, mo = oracle.extract(imgs[i], oracle.params(1000))
        n = int(cnt[i, 0])
        _assert_kps_equal(kps[i, :n], desc[i, :n], int(cnt[i, 1]), ko, do, mo, f"batch frame {i}")


def test_error_contract(gpu_lib):
    from mam3slam_amd._lib import MAM_ERR_EMPTY

    ext = _extractor(1000)
    k, d, m = ext(np.zeros((0, 0), np.uint8))
    assert m == MAM_ERR_EMPTY and len(k) == 0
    # flat image: no corners at all -> zero keypoints, monoIndex 0
    k, d, m = ext(np.full((480, 640), 128, np.uint8))
    assert len(k) == 0 and m == 0


@pytest.mark.parametrize("w,h,nfeat", CASES[:3])
def test_batch_pyramid_levels(gpu_lib, oracle, w, h, nfeat):
    """Batches (> 4 frames) take the per-level one-thread-per-quad resize (k_pyr_flat), single frames the one-launch
    band pyramid: both bit-exact vs cv::resize's fixed-point restatement on every level and frame."""
    import torch

    F = 6
    ext = _extractor(nfeat)
    imgs = np.stack([synth.make_frame(w, h, agent=6, frame=i) for i in range(F)])
    cap = ext.max_keypoints()
    d_img = torch.from_numpy(imgs).cuda()
    d_kps = torch.zeros((F, cap * 28), dtype=torch.uint8, device="cuda")
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros((F, 2), dtype=torch.int32, device="cuda")
    ext.extract_batch_device(d_img.data_ptr(), F, w, h, w, w * h, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                             d_cnt.data_ptr())
    torch.cuda.synchronize()
    p = oracle.params(nfeat)
    for i in (0, F - 1):
        levels = oracle.pyramid(imgs[i], p)
        for l, lev in enumerate(levels):
            d = _first_diff(ext.level(l, i), lev)
            assert d is None, f"frame {i} level {l} pixel {d}"
            d = _first_diff(ext.debug_blurred(l, i), oracle.gaussian7(lev))
            assert d is None, f"frame {i} blurred level {l} pixel {d}"


def test_batch_input_ends_at_last_row(gpu_lib, oracle):
    """The caller's frames end exactly at the last row of the last frame (a 2 MiB-multiple device allocation with no
    allocator slack): the word-wise level-0 reads of the batched resize must stay inside it (k_pyr_flat reads whole
    source words; the words past a row are zero-weight edge columns). 4 frames of 1024 x 512 = exactly 2 MiB."""
    import torch

    w, h, F = 1024, 512, 4
    ext = _extractor(1000)
    imgs = np.stack([synth.make_frame(w, h, agent=8, frame=i) for i in range(F)])
    cap = ext.max_keypoints()
    d_img = torch.empty(F * w * h, dtype=torch.uint8, device="cuda")
    assert d_img.untyped_storage().nbytes() == 2 * 1024 * 1024
    d_img.copy_(torch.from_numpy(imgs.reshape(-1)))
    d_kps = torch.zeros((F, cap * 28), dtype=torch.uint8, device="cuda")
    d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device="cuda")
    d_cnt = torch.zeros((F, 2), dtype=torch.int32, device="cuda")
    ext.extract_batch_device(d_img.data_ptr(), F, w, h, w, w * h, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                             d_cnt.data_ptr())
    torch.cuda.synchronize()
    levels = oracle.pyramid(imgs[F - 1], oracle.params(1000))
    for l, lev in enumerate(levels):
        assert _first_diff(ext.level(l, F - 1), lev) is None, f"level {l}"
    ko, do, _ = oracle.extract(imgs[F - 1], oracle.params(1000))
    n = int(d_cnt[F - 1, 0])
    assert n == len(ko) and np.array_equal(d_desc[F - 1, :n].cpu().numpy(), do)


@pytest.mark.parametrize("nt", [0, 256, 512, 1024])
def test_distribute_widths_bit_exact(gpu_lib, oracle, nt):
    """Every DistributeOctTree kernel width (k_distribute2 at 256 / 512 / 1024 threads, the round-3 kernel) gives the
    oracle's keypoints in the oracle's order, single frames and a 3-frame batch, on every extractor shape (incl. the
    5x init extractor, whose final phase sorts more than 256 candidates)."""
    import torch

    from mam3slam_amd.orb import KP_DTYPE

    for w, h, nfeat in CASES:
        ext = _extractor(nfeat)
        ext.set_distribute_threads(nt)
        p = oracle.params(nfeat)
        imgs = np.stack([synth.make_frame(w, h, agent=5, frame=i) for i in range(3)])
        ref = [oracle.extract(imgs[i], p) for i in range(3)]
        kg, dg, mg = ext(imgs[0])
        _assert_kps_equal(kg, dg, mg, *ref[0], f"nt {nt} {w}x{h}/{nfeat} single")
        cap = ext.max_keypoints()
        d_img = torch.from_numpy(imgs).cuda()
        d_kps = torch.zeros((3, cap * 28), dtype=torch.uint8, device="cuda")
        d_desc = torch.zeros((3, cap, 32), dtype=torch.uint8, device="cuda")
        d_cnt = torch.zeros((3, 2), dtype=torch.int32, device="cuda")
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        ext.extract_batch_device(d_img.data_ptr(), 3, w, h, w, w * h, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                                 d_cnt.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
        cnt = d_cnt.cpu().numpy()
        kps = d_kps.cpu().numpy().view(KP_DTYPE).reshape(3, cap)
        desc = d_desc.cpu().numpy()
        for i in range(3):
            n = int(cnt[i, 0])
            _assert_kps_equal(kps[i, :n], desc[i, :n], int(cnt[i, 1]), *ref[i], f"nt {nt} {w}x{h}/{nfeat} batch {i}")
        ext.close()


@pytest.mark.parametrize("fork", [0, 1])
def test_latency_mode_fork_bit_exact(gpu_lib, oracle, fork):
    """The latency mode's three-stream dataflow (level 0's FAST + DistributeOctTree beside the pyramid, the blur beside
    the other levels) and the in-order single stream give the oracle's output: through the host API, and at B = 1 on a
    device stream captured into a HIP graph (the fork / join events inside the capture) and replayed."""
    import torch

    from mam3slam_amd.orb import KP_DTYPE

    for w, h, nfeat in CASES[:3]:
        ext = _extractor(nfeat)
        ext.set_fork(fork)
        p = oracle.params(nfeat)
        imgs = [synth.make_frame(w, h, agent=6, frame=i) for i in range(2)]
        ref = [oracle.extract(im, p) for im in imgs]
        for i in range(2):
            kg, dg, mg = ext(imgs[i])
            _assert_kps_equal(kg, dg, mg, *ref[i], f"fork {fork} {w}x{h}/{nfeat} host {i}")
        cap = ext.max_keypoints()
        d_img = torch.from_numpy(imgs[0]).cuda()
        d_kps = torch.zeros(cap * 28, dtype=torch.uint8, device="cuda")
        d_desc = torch.zeros((cap, 32), dtype=torch.uint8, device="cuda")
        d_cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            ext.extract_batch_device(d_img.data_ptr(), 1, w, h, w, w * h, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                                     d_cnt.data_ptr(), stream=st.cuda_stream)
        for i in (1, 0):
            d_img.copy_(torch.from_numpy(imgs[i]))
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            n = int(d_cnt[0])
            kps = d_kps.cpu().numpy().view(KP_DTYPE)[:n]
            _assert_kps_equal(kps, d_desc.cpu().numpy()[:n], int(d_cnt[1]), *ref[i], f"fork {fork} {w}x{h} graph {i}")
        ext.close()


@pytest.mark.parametrize("w,h,nfeat", CASES[:3])
def test_fast_chunks_bit_exact(gpu_lib, oracle, w, h, nfeat):
    """k_fast_chunks (FAST over chunks of up to 4 cells of a cell row: one staging and one strength map per chunk, NMS
    with the other cells' pixels masked, per-cell threshold choice and ordered emit) gives the oracle's per-level
    candidates and the end-to-end output, single frames (latency mode) and a batch."""
    ext = _extractor(nfeat)
    ext.set_fast_chunks(1)
    p = oracle.params(nfeat)
    for fr in range(2):
        img = synth.make_frame(w, h, agent=7, frame=fr)
        kg, dg, mg = ext(img)
        ko, do, mo = oracle.extract(img, p)
        _assert_kps_equal(kg, dg, mg, ko, do, mo, f"chunks {w}x{h}/{nfeat} frame {fr}")
        for l in range(8):
            cand_o, _ = oracle.level_stage(img, l, p)
            cand_g = ext.debug_candidates(l)
            assert len(cand_g) == len(cand_o), f"level {l}: {len(cand_g)} candidates vs oracle {len(cand_o)}"
            d = _first_diff(cand_g, cand_o)
            assert d is None, f"level {l} candidate {d}: gpu={oracle.unpack(cand_g[d])} oracle={oracle.unpack(cand_o[d])}"
    ext.set_fork(0)   # one stream, every level in one launch
    img = synth.make_frame(w, h, agent=7, frame=5)
    kg, dg, mg = ext(img)
    _assert_kps_equal(kg, dg, mg, *oracle.extract(img, p), f"chunks {w}x{h}/{nfeat} no fork")
    ext.close()


@pytest.mark.parametrize("fb", [0, 1])
def test_fast_blur_launch_bit_exact(gpu_lib, oracle, fb):
    """FAST and the blur in one launch (k_fast_blur, the latency-mode default) or in two (k_blur7 + k_fast_cells):
    the oracle's keypoints, descriptors and blurred levels either way, single frames through the host API and a
    device batch of 3 frames."""
    import torch

    from mam3slam_amd.orb import KP_DTYPE

    for w, h, nfeat in CASES[:3]:
        ext = _extractor(nfeat)
        ext.set_fast_blur(fb)
        p = oracle.params(nfeat)
        imgs = np.stack([synth.make_frame(w, h, agent=8, frame=i) for i in range(3)])
        for i in range(2):
            kg, dg, mg = ext(imgs[i])
            _assert_kps_equal(kg, dg, mg, *oracle.extract(imgs[i], p), f"fast_blur {fb} {w}x{h}/{nfeat} frame {i}")
        levels = oracle.pyramid(imgs[1], p)
        for l in (0, 3, 7):
            d = _first_diff(ext.debug_blurred(l), oracle.gaussian7(levels[l]))
            assert d is None, f"fast_blur {fb} {w}x{h} blurred level {l} pixel {d}"
        F = 3
        cap = ext.max_keypoints()
        d_img = torch.from_numpy(imgs).cuda()
        d_kps = torch.zeros((F, cap * 28), dtype=torch.uint8, device="cuda")
        d_desc = torch.zeros((F, cap, 32), dtype=torch.uint8, device="cuda")
        d_cnt = torch.zeros((F, 2), dtype=torch.int32, device="cuda")
        ext.extract_batch_device(d_img.data_ptr(), F, w, h, w, w * h, d_kps.data_ptr(), d_desc.data_ptr(), cap,
                                 d_cnt.data_ptr())
        torch.cuda.synchronize()
        for i in range(F):
            n = int(d_cnt[i, 0])
            kps = d_kps[i].cpu().numpy().view(KP_DTYPE)[:n]
            _assert_kps_equal(kps, d_desc[i].cpu().numpy()[:n], int(d_cnt[i, 1]), *oracle.extract(imgs[i], p),
                              f"fast_blur {fb} {w}x{h}/{nfeat} batch {i}")
        ext.close()


def test_large_extractor_distribute_fallback(gpu_lib, oracle):
    """A 10000-feature extractor at 1280x720 (Tracking.cc:606's 5x init extractor for 2000 features): level 0's
    DistributeOctTree needs more LDS than the 1024-thread k_distribute2 has, so the narrower width (or the round-3
    kernel) runs instead of the geometry being refused — bit-exact against the oracle, single frame and batch."""
    from mam3slam_amd import ORBextractor

    ext = ORBextractor(10000, 1.2, 8, 20, 7)
    img = synth.make_frame(1280, 720, agent=9, frame=4)
    kg, dg, mg = ext(img)
    ko, do, mo = oracle.extract(img, oracle.params(10000))
    _assert_kps_equal(kg, dg, mg, ko, do, mo, "10000 features")
    assert len(kg) > 5000
