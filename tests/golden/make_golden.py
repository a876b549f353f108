"""Generate the golden fixtures under tests/golden/ (run from the repo root: python tests/golden/make_golden.py).

The reference cannot be built or imported here and ships no golden vectors, so these fixtures are
produced by the CPU oracle (oracle/, a line-by-line restatement of the reference path) on seeded synthetic inputs,
and stored WITH the inputs so nothing has to be regenerated to check them:

  orb.npz    3 frames (2 x 320x240 / 500 features, 1 x 640x480 / 1000 features): keypoints (cv::KeyPoint layout),
             descriptors, monoIndex of ORBextractor::operator()
  match.npz  one SearchByProjection(F, vpMapPoints) case, one SearchByProjection(Cur, Last) case and one
             SearchForTriangulation case: flattened inputs + the oracle's per-keypoint outputs and match counts
  lba.npz    a 6-KF / 120-point LocalBundleAdjustment problem + the oracle's poses, points, per-edge chi2,
             iterations and Levenberg trials

tests/test_golden.py pins the oracle to these files (CPU) and checks the GPU path against them (-m gpu).
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.dirname(os.path.abspath(__file__))

ORB_CASES = [(320, 240, 500, 11, 0), (320, 240, 500, 12, 3), (640, 480, 1000, 13, 1)]


def make_orb(oracle, synth):
    out = {}
    for i, (w, h, nf, agent, fr) in enumerate(ORB_CASES):
        img = synth.make_frame(w, h, agent=agent, frame=fr)
        k, d, m = oracle.extract(img, oracle.params(nf))
        out[f"img{i}"] = img
        out[f"nfeat{i}"] = np.int32(nf)
        out[f"kps{i}"] = k.view(np.uint8).reshape(len(k), 28)
        out[f"desc{i}"] = d
        out[f"mono{i}"] = np.int32(m)
    np.savez_compressed(os.path.join(OUT, "orb.npz"), **out)


def flat_featvec(fv):
    from mam3slam_amd.match import flatten_featvec

    ids, off, feats = flatten_featvec(fv)
    return ids, off, feats


def make_match(oracle, synth, scene):
    w, h = 640, 480
    img = synth.make_frame(w, h, agent=21, frame=2)
    k, d, _ = oracle.extract(img, oracle.params(1000))
    out = {"w": np.int32(w), "h": np.int32(h)}
    # local map search, th 3, nnratio 0.8, 10% keypoints pre-taken
    rng = np.random.default_rng(401)
    F = scene.make_frame_data(k, d, w, h, rng, taken_frac=0.1)
    mps = scene.local_mappoints(F, rng)
    n, o = oracle.search_by_projection(F, mps, 3.0, False, 50.0, 0.8)
    out.update(local_keys=F.keys.view(np.uint8).reshape(-1, 28), local_desc=F.desc, local_taken=F.taken,
               local_mps=mps.view(np.uint8).reshape(len(mps), -1), local_out=o, local_n=np.int32(n))
    # motion-model search, th 15, rotation check on
    rng = np.random.default_rng(402)
    F = scene.make_frame_data(k, d, w, h, rng, taken_frac=0.05)
    F.pose = scene.small_pose(rng)
    cam = scene.pinhole(w, h)
    last = scene.motion_last_frame(F, cam, rng)
    n, o = oracle.search_by_projection_motion(F, last, cam, 15.0, True)
    out.update(motion_keys=F.keys.view(np.uint8).reshape(-1, 28), motion_desc=F.desc, motion_taken=F.taken,
               motion_q=np.asarray(F.pose[0], np.float32), motion_t=np.asarray(F.pose[1], np.float32),
               motion_last=last.view(np.uint8).reshape(len(last), -1), motion_out=o, motion_n=np.int32(n))
    # SearchForTriangulation, nnratio 0.6, no orientation check, fine epipolar test
    rng = np.random.default_rng(403)
    F = scene.make_frame_data(k, d, w, h)
    KF1, KF2, F12, ep = scene.keyframe_pair(F, cam, rng)
    n, o = oracle.search_for_triangulation(KF1, KF2, F12, ep, False, False)
    i1, o1, f1 = flat_featvec(KF1.featvec)
    i2, o2, f2 = flat_featvec(KF2.featvec)
    out.update(tri_keys1=KF1.keys.view(np.uint8).reshape(-1, 28), tri_desc1=KF1.desc, tri_has1=KF1.has_mp,
               tri_keys2=KF2.keys.view(np.uint8).reshape(-1, 28), tri_desc2=KF2.desc, tri_has2=KF2.has_mp,
               tri_ids1=i1, tri_off1=o1, tri_feats1=f1, tri_ids2=i2, tri_off2=o2, tri_feats2=f2,
               tri_F12=F12, tri_ep=ep, tri_out=o, tri_n=np.int32(n))
    np.savez_compressed(os.path.join(OUT, "match.npz"), **out)


def make_lba(oracle):
    from mam3slam_amd.lba import synthetic_problem

    prob = synthetic_problem(n_opt=6, n_fixed=2, n_points=120, obs_per_point=4, seed=31, outlier_frac=0.08)
    r = oracle.lba_solve(prob)
    out = {f"p_{k}": getattr(prob, k) for k in ("pose_id", "pose_fixed", "pose_q", "pose_t", "point_id", "point_xyz",
                                                   "edge_point", "edge_pose", "edge_obs", "edge_inv_sigma2", "cams")}
    out.update(r_pose_q=r.pose_q, r_pose_t=r.pose_t, r_point_xyz=r.point_xyz, r_edge_chi2=r.edge_chi2,
               r_edge_depth_ok=r.edge_depth_ok, r_iterations=np.int32(r.iterations), r_trials=np.int32(r.lm_trials),
               r_initial_chi2=np.float64(r.initial_chi2), r_final_chi2=np.float64(r.final_chi2))
    np.savez_compressed(os.path.join(OUT, "lba.npz"), **out)


def main():
    from mam3slam_amd import scene, synth
    from oracle import oracle_py

    oracle_py.build()
    make_orb(oracle_py, synth)
    make_match(oracle_py, synth, scene)
    make_lba(oracle_py)
    for f in ("orb.npz", "match.npz", "lba.npz"):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
