"""ORBVocabulary — Python mirror of DBoW2::TemplatedVocabulary<FORB> (ORB-SLAM3's ORBVocabulary) over the C-ABI
(include/mam_bow.h): the tree descent of every feature runs on gfx950, the BowVector / FeatureVector maps are built
here exactly as DBoW2 builds them.

Reference interface (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h):
    bool loadFromTextFile(const std::string&)                                  :1338-1420
    void saveToTextFile(const std::string&) const                              :1429-1449
    void transform(const vector<TDescriptor>&, BowVector&, FeatureVector&, int levelsup) const   :1125-1192
as used by KeyFrame::ComputeBoW / Frame::ComputeBoW (levelsup = 4). BowVector = {word id: value} (std::map order),
FeatureVector = {node id: [feature indices]}.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import MamError, check, lib

TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3                                    # WeightingType
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)  # ScoringType

_SIGS = {
    "mam_bow_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    "mam_bow_destroy": (None, [C.c_void_p]),
    "mam_bow_words": (C.c_int, [C.c_void_p]),
    "mam_bow_transform": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_bow_transform_batch_device": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mam_bow_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "mam_bow_stage_times": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
}


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _bind():
    L = lib()
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    return L


class VocabularyArrays:
    """The tree as the text format lists it: node 0 = root, nodes 1.. in file order with parent, leaf flag,
    32-byte descriptor and weight."""

    def __init__(self, k, L, scoring, weighting, parent, is_leaf, desc, weight):
        self.k, self.L, self.scoring, self.weighting = int(k), int(L), int(scoring), int(weighting)
        self.parent = np.ascontiguousarray(parent, np.int32)
        self.is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        self.desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        self.weight = np.ascontiguousarray(weight, np.float64)
        n = len(self.parent)
        if not (len(self.is_leaf) == n and len(self.desc) == n and len(self.weight) == n):
            raise MamError("vocabulary arrays must all have n_nodes rows")

    @property
    def n_nodes(self):
        return len(self.parent)


def load_from_text_file(path: str) -> VocabularyArrays:
    """loadFromTextFile (TemplatedVocabulary.h:1338-1420): header "k L scoring weighting", then one node per line
    "parent isLeaf d0 .. d31 weight". Empty lines are skipped (the reference's loop turns a trailing empty line into
    a node built from unread values)."""
    with open(path) as f:
        head = f.readline().split()
        k, L, n1, n2 = (int(x) for x in head[:4])
        if k < 0 or k > 20 or L < 1 or L > 10 or n1 < 0 or n1 > 5 or n2 < 0 or n2 > 3:
            raise MamError("Vocabulary loading failure: This is not a correct text file!")
        rows = [ln.split() for ln in f if ln.strip()]
    n = len(rows) + 1
    parent = np.zeros(n, np.int32)
    leaf = np.zeros(n, np.uint8)
    desc = np.zeros((n, 32), np.uint8)
    weight = np.zeros(n, np.float64)
    for i, r in enumerate(rows, start=1):
        parent[i] = int(r[0])
        leaf[i] = 1 if int(r[1]) > 0 else 0
        desc[i] = [int(x) & 0xFF for x in r[2:34]]
        weight[i] = float(r[34])
    return VocabularyArrays(k, L, n1, n2, parent, leaf, desc, weight)


def save_to_text_file(v: VocabularyArrays, path: str) -> None:
    """saveToTextFile (TemplatedVocabulary.h:1429-1449); a node is written as a leaf iff it has no children."""
    has_child = np.zeros(v.n_nodes, bool)
    has_child[v.parent[1:]] = True
    with open(path, "w") as f:
        f.write(f"{v.k} {v.L}  {v.scoring} {v.weighting}\n")
        for i in range(1, v.n_nodes):
            d = " ".join(str(int(x)) for x in v.desc[i])
            f.write(f"{v.parent[i]} {0 if has_child[i] else 1} {d}  {repr(float(v.weight[i]))}\n")


def synthetic_vocabulary(k=10, L=6, rng=None, early_leaf=0.05, stopped=0.02, min_leaf_depth=2) -> VocabularyArrays:
    """A k-ary vocabulary tree of depth L (there is no ORBvoc.txt here): every child descriptor is its parent's with
    bits flipped (fewer deeper down, as k-means centroids refine), some nodes become leaves early (at depth >=
    min_leaf_depth), leaf weights are idf-like positive values with a few stopped (0) words. Nodes are numbered
    breadth-first, children contiguous, as DBoW2's HKmeansStep creates them."""
    rng = np.random.default_rng(0) if rng is None else rng
    parent = [np.zeros(1, np.int32)]
    desc = [rng.integers(0, 256, (1, 32), dtype=np.uint8)]
    leaf = [np.zeros(1, np.uint8)]
    level_ids = np.array([0])
    n = 1
    for depth in range(1, L + 1):
        expand = level_ids
        if depth > min_leaf_depth:
            keep = rng.random(len(expand)) >= early_leaf
            keep[0] = True
            expand = expand[keep]
        m = len(expand) * k
        par = np.repeat(expand, k).astype(np.int32)
        base = np.concatenate(desc)[par]
        flips = rng.integers(0, 256, (m, 32), dtype=np.uint8)
        for _ in range(min(depth, 3)):   # bit probability 1/2, 1/4, 1/8 per level
            flips &= rng.integers(0, 256, (m, 32), dtype=np.uint8)
        parent.append(par)
        desc.append(base ^ flips)
        leaf.append(np.full(m, 1 if depth == L else 0, np.uint8))
        level_ids = np.arange(n, n + m)
        n += m
    parent = np.concatenate(parent)
    desc = np.concatenate(desc)
    leaf = np.concatenate(leaf)
    has_child = np.zeros(n, bool)
    has_child[parent[1:]] = True
    leaf = (~has_child).astype(np.uint8)
    leaf[0] = 0
    weight = np.where(leaf == 1, rng.uniform(0.5, 9.0, n), 0.0)
    weight[(leaf == 1) & (rng.random(n) < stopped)] = 0.0
    return VocabularyArrays(k, L, L1_NORM, TF_IDF, parent, leaf, desc, weight)


def bow_from_words(words, weights, nids, weighting=TF_IDF, scoring=L1_NORM):
    """The maps of transform(features, v, fv, levelsup) (TemplatedVocabulary.h:1125-1192, BowVector.cpp:34-84,
    FeatureVector.cpp:31-45) from the per-feature descent results: stopped words (weight 0) skipped, weights summed
    per word in feature order (TF / TF_IDF) or the first kept (IDF / BINARY), then the scoring's normalisation."""
    bow: dict = {}
    fv: dict = {}
    for i, (w, x, nid) in enumerate(zip(words.tolist(), weights.tolist(), nids.tolist())):
        if not x > 0:
            continue
        if weighting in (TF_IDF, TF):
            bow[w] = bow[w] + x if w in bow else x
        elif w not in bow:
            bow[w] = x
        fv.setdefault(nid, []).append(i)
    must = scoring != DOT_PRODUCT
    if weighting in (TF_IDF, TF) and bow and not must:
        nd = float(len(bow))
        bow = {w: x / nd for w, x in bow.items()}
    if must:
        keys = sorted(bow)
        if scoring == L2_NORM:
            norm = 0.0
            for w in keys:
                norm += bow[w] * bow[w]
            norm = float(np.sqrt(norm))
        else:
            norm = 0.0
            for w in keys:
                norm += abs(bow[w])
        if norm > 0.0:
            bow = {w: bow[w] / norm for w in keys}
    return dict(sorted(bow.items())), dict(sorted(fv.items()))


class ORBVocabulary:
    """ORBVocabulary on the GPU. `v`: VocabularyArrays (load_from_text_file / synthetic_vocabulary)."""

    def __init__(self, v: VocabularyArrays, device: int = 0):
        self.v = v
        self._L = _bind()
        self._h = C.c_void_p()
        check(self._L.mam_bow_create(int(device), v.k, v.L, v.weighting, v.scoring, v.n_nodes, _p(v.parent),
                                     _p(v.is_leaf), _p(v.desc), _p(v.weight), C.byref(self._h)), "mam_bow_create")

    @classmethod
    def loadFromTextFile(cls, path: str, device: int = 0) -> "ORBVocabulary":
        return cls(load_from_text_file(path), device)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._L.mam_bow_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def size(self) -> int:
        return int(self._L.mam_bow_words(self._h))

    def transform_features(self, descs: np.ndarray, levelsup: int = 4):
        """Per feature: (word id, weight, node at level L - levelsup) — transform(feature, id, w, &nid, levelsup)."""
        d = np.ascontiguousarray(descs, np.uint8).reshape(-1, 32)
        n = len(d)
        w = np.zeros(max(n, 1), np.uint32)
        x = np.zeros(max(n, 1), np.float64)
        nid = np.zeros(max(n, 1), np.uint32)
        check(self._L.mam_bow_transform(self._h, n, _p(d), int(levelsup), _p(w), _p(x), _p(nid)), "bow_transform")
        return w[:n], x[:n], nid[:n]

    def transform(self, descs: np.ndarray, levelsup: int = 4):
        """transform(features, BowVector, FeatureVector, levelsup) -> (bow {word: value}, featvec {node: [i]})."""
        w, x, nid = self.transform_features(descs, levelsup)
        return bow_from_words(w, x, nid, self.v.weighting, self.v.scoring)

    def transform_batch_device(self, nframes: int, d_desc: int, desc_stride: int, d_counts: int, levelsup: int,
                               d_word: int, d_weight: int, d_nid: int, stream: int = 0):
        return check(self._L.mam_bow_transform_batch_device(
            self._h, int(nframes), C.c_void_p(d_desc), int(desc_stride), C.c_void_p(d_counts), int(levelsup),
            C.c_void_p(d_word), C.c_void_p(d_weight), C.c_void_p(d_nid), C.c_void_p(stream)), "bow_transform_batch")

    def set_profiling(self, enable: bool):
        check(self._L.mam_bow_set_profiling(self._h, 1 if enable else 0), "bow_set_profiling")

    def stage_times(self):
        ms = np.zeros(1, np.float64)
        n = np.zeros(1, np.int64)
        check(self._L.mam_bow_stage_times(self._h, _p(ms), _p(n)), "bow_stage_times")
        return {"transform": (float(ms[0]), int(n[0]))}
