"""GPU parity: DBoW2 vocabulary transform (TemplatedVocabulary.h:1125-1259) on the HIP path vs the CPU oracle —
bit-exact word ids, weights and FeatureVector nodes per feature, identical BowVector / FeatureVector maps.

There is no ORBvoc.txt here (.MISSING_LARGE_BLOBS): the trees are synthetic (bow.synthetic_vocabulary: k-ary,
children refined from their parent's descriptor, early leaves, stopped words), written to and read back from the
reference's text format. Features are real ORB descriptors plus random ones.
"""
import numpy as np
import pytest

from mam3slam_amd import bow, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def descs(oracle):
    out = []
    for fr in range(2):
        img = synth.make_frame(1280, 720, agent=2, frame=fr)
        _, d, _ = oracle.extract(img, oracle.params(2000))
        out.append(d)
    out.append(np.random.default_rng(3).integers(0, 256, (700, 32), dtype=np.uint8))
    return out


@pytest.mark.parametrize("k,L,levelsup", [(10, 4, 2), (10, 6, 4), (7, 5, 4), (16, 3, 1), (20, 3, 4), (5, 4, 0)])
def test_bow_transform(gpu_lib, oracle, descs, tmp_path, k, L, levelsup):
    rng = np.random.default_rng(k * 100 + L)
    v = bow.synthetic_vocabulary(k, L, rng, early_leaf=0.1)
    path = tmp_path / "voc.txt"
    bow.save_to_text_file(v, str(path))
    voc = bow.ORBVocabulary.loadFromTextFile(str(path))
    assert voc.size() == int(v.is_leaf.sum())
    for d in descs:
        w, x, nid = voc.transform_features(d, levelsup)
        (wo, xo, nido), Bo, Fo = oracle.bow_transform(voc.v, d, levelsup)
        assert np.array_equal(w, wo) and np.array_equal(x, xo) and np.array_equal(nid, nido)
        B, F = voc.transform(d, levelsup)
        assert B == Bo and F == Fo   # exact doubles: same summation and normalisation order
        assert (len(F) > 1 or L - levelsup <= 0) and abs(sum(B.values()) - 1.0) < 1e-12


def test_bow_edges(gpu_lib, oracle, descs):
    rng = np.random.default_rng(5)
    v = bow.synthetic_vocabulary(10, 3, rng, stopped=0.5)   # half the words stopped
    voc = bow.ORBVocabulary(v)
    d = descs[0]
    (wo, xo, nido), Bo, Fo = oracle.bow_transform(v, d, 4)
    w, x, nid = voc.transform_features(d, 4)
    assert np.array_equal(w, wo) and np.array_equal(x, xo) and np.array_equal(nid, nido)
    assert (x == 0).any() and voc.transform(d, 4) == (Bo, Fo)
    # no features; ties: a feature equal to two sibling centroids takes the first
    assert voc.transform(d[:0], 4) == ({}, {})
    v2 = bow.synthetic_vocabulary(4, 2, rng)
    v2.desc[2] = v2.desc[1]
    voc2 = bow.ORBVocabulary(v2)
    feat = np.repeat(v2.desc[1][None], 3, 0)
    (wo, xo, nido), _, _ = oracle.bow_transform(v2, feat, 1)
    w, x, nid = voc2.transform_features(feat, 1)
    assert np.array_equal(w, wo) and np.array_equal(nid, nido) and (nid == 1).all()


def test_bow_batch_device(gpu_lib, oracle, descs):
    import torch

    v = bow.synthetic_vocabulary(10, 5, np.random.default_rng(9))
    voc = bow.ORBVocabulary(v)
    B = len(descs)
    S = max(len(d) for d in descs)
    D = np.zeros((B, S, 32), np.uint8)
    cnt = np.zeros((B, 2), np.int32)
    for f, d in enumerate(descs):
        D[f, :len(d)] = d
        cnt[f, 0] = len(d)
    dev = torch.device("cuda")
    t_d, t_c = torch.from_numpy(D).to(dev), torch.from_numpy(cnt).to(dev)
    t_w = torch.zeros((B, S), dtype=torch.int32, device=dev)
    t_x = torch.zeros((B, S), dtype=torch.float64, device=dev)
    t_n = torch.zeros((B, S), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    voc.transform_batch_device(B, t_d.data_ptr(), S, t_c.data_ptr(), 4, t_w.data_ptr(), t_x.data_ptr(), t_n.data_ptr())
    torch.cuda.synchronize()
    gw, gx, gn = t_w.cpu().numpy().view(np.uint32), t_x.cpu().numpy(), t_n.cpu().numpy().view(np.uint32)
    for f, d in enumerate(descs):
        (wo, xo, nido), _, _ = oracle.bow_transform(v, d, 4)
        n = len(d)
        assert np.array_equal(gw[f, :n], wo) and np.array_equal(gx[f, :n], xo) and np.array_equal(gn[f, :n], nido)


def test_triangulation_on_bow_feature_vectors(gpu_lib, oracle):
    """SearchForTriangulation (a15) walking FeatureVectors made by the GPU transform (levelsup 4, as
    KeyFrame::ComputeBoW), GPU search vs oracle search — the LocalMapping chain ComputeBoW -> CreateNewMapPoints."""
    from mam3slam_amd import scene
    from mam3slam_amd.match import ORBmatcher

    img = synth.make_frame(640, 480, agent=6, frame=1)
    k, d, _ = oracle.extract(img, oracle.params(1000))
    rng = np.random.default_rng(21)
    F = scene.make_frame_data(k, d, 640, 480)
    KF1, KF2, F12, ep = scene.keyframe_pair(F, scene.pinhole(640, 480), rng)
    voc = bow.ORBVocabulary(bow.synthetic_vocabulary(10, 6, np.random.default_rng(4), early_leaf=0.02))
    KF1.featvec = voc.transform(KF1.desc, 4)[1]
    KF2.featvec = voc.transform(KF2.desc, 4)[1]
    assert len(KF1.featvec) > 20
    for coarse in (False, True):
        ng, pg = ORBmatcher(0.6, True).SearchForTriangulation(KF1, KF2, F12, ep, False, coarse)
        no, oo = oracle.search_for_triangulation(KF1, KF2, F12, ep, True, coarse)
        idx = np.nonzero(oo >= 0)[0]
        assert ng == no and np.array_equal(pg, np.stack([idx, oo[idx]], 1)), coarse
