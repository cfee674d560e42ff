"""Ideal features for the tracking loop (test infrastructure): landmarks on the rendered room's
surfaces, each with a fixed random 256-d descriptor, projected into a frame with its ground-truth
pose (sub-pixel noise, small descriptor noise, occlusion test against the rendered depth).  With
such correspondences the reference's pipeline (Slam::process_frame, Slam.cpp:809-1135) must follow
the synthetic trajectory; tests use them to separate "random SuperPoint weights" from a
restatement error in the tracker (host/tracker.hpp)."""
import numpy as np

import synth

K = synth.K_TUM
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4"), ("class_id", "<i4")])


def landmarks(frames, n_land=4000, seed=11):
    """Landmark positions P [L][3] (world) back-projected from random pixels of the frames (dicts
    with depth, R_wc, t_wc) and unit descriptors D [L][256]."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = K
    pts = []
    per = n_land // len(frames)
    for f in frames:
        u = rng.uniform(0, 639, per)
        v = rng.uniform(0, 479, per)
        z = f["depth"][np.round(v).astype(int), np.round(u).astype(int)].astype(np.float64)
        ok = (z > 0.3) & (z < 4.5)
        pc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)[ok]
        pts.append(pc @ f["R_wc"].T + f["t_wc"])
    P = np.concatenate(pts)
    D = rng.standard_normal((len(P), 256)).astype(np.float32)
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    return P, D


def visible(f, P):
    """Indices of the landmarks frame f sees unoccluded, and their exact projections."""
    fx, fy, cx, cy = K
    pc = (P - f["t_wc"]) @ f["R_wc"]
    z = pc[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        u = fx * pc[:, 0] / z + cx
        v = fy * pc[:, 1] / z + cy
    vis = (z > 0.2) & (u >= 1) & (u < 638) & (v >= 1) & (v < 478)
    idx = np.nonzero(vis)[0]
    dz = f["depth"][np.round(v[idx]).astype(int), np.round(u[idx]).astype(int)]
    idx = idx[np.abs(dz - z[idx]) < 0.03]
    return idx, u, v


def features(f, P, D, rng, pick=None, cap=400):
    """(keypoints, descriptors, landmark ids) of frame f: `pick` (landmark ids, default every
    visible one) shuffled and capped at cap, with 0.3 px / 0.02 descriptor noise."""
    idx, u, v = visible(f, P)
    if pick is not None:
        idx = np.intersect1d(idx, np.asarray(pick))
    idx = idx[rng.permutation(len(idx))[:cap]]
    k = np.zeros(len(idx), KP_DTYPE)
    k["x"] = u[idx] + rng.normal(0, 0.3, len(idx))
    k["y"] = v[idx] + rng.normal(0, 0.3, len(idx))
    k["size"], k["angle"], k["response"], k["class_id"] = 8.0, -1.0, 0.5, -1
    d = D[idx] + rng.normal(0, 0.02, (len(idx), 256)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return k, d.astype(np.float32), idx


def loop_frames(L):
    return [dict(depth=L["depth"][i], R_wc=L["R_wc"][i], t_wc=L["t_wc"][i]) for i in range(len(L["depth"]))]


def recovery_sequence(L, n_frames, k_jump, seed=13, n_land=20000):
    """Ideal features along the closed loop (frame g uses rendered frame g mod U) in which frame
    k_jump (second lap or later) sees only landmarks that the previous 12 frames did not observe
    but that the same place's frames one lap earlier did: ratio matching against the reference
    keyframe and the last frame finds nothing (< MIN_MATCHES), matching against the map does, so
    Slam::try_pnp_recovery (Slam.cpp:535-613) must recover the pose.  Returns (feats, P)."""
    U = len(L["depth"])
    fr = loop_frames(L)
    P, D = landmarks(fr, n_land=n_land)
    rng = np.random.default_rng(seed)
    feats, ids = [], []
    for g in range(n_frames):
        f = fr[g % U]
        if g == k_jump:
            assert g >= U + 3
            seen_recent = np.unique(np.concatenate(ids[g - 12:g]))
            seen_lap = np.unique(np.concatenate(ids[g - U - 3:g - U + 4]))
            pick = np.setdiff1d(seen_lap, seen_recent)
            k, d, i = features(f, P, D, rng, pick=pick)
        else:
            k, d, i = features(f, P, D, rng)
        feats.append((k, d))
        ids.append(i)
    return feats, P


class NoisySequence:
    """Realistic-noise features along the closed loop (a known-answer run that
    is neither ideal nor random-weight): every landmark has a fixed saliency and a frame keeps its
    400 most salient visible landmarks (saliency jittered per frame), so detections repeat across
    frames as a trained detector's do; then

    * keypoints carry `px` pixels of Gaussian position noise;
    * descriptors carry `desc_noise` per dimension of Gaussian noise (unit 256-d vectors: 0.03 puts
      a true pair at ~0.68 against ~1.41 for unrelated landmarks, before the ratio test);
    * a fraction `shuffle` of each frame's keypoints carry the descriptor of another of its own
      keypoints (a random derangement among them), independently per frame, so ratio matching
      between two frames yields confidently wrong pairs (outliers for F / 3D-3D / PnP);
    * the depth image loses a fraction `dropout` of its pixels (0 = invalid, Frame.cpp:51-52).

    frame(g) returns (keypoints, descriptors, depth, landmark ids, wrong) for processed frame g
    (rendered frame g mod U); wrong marks the keypoints whose descriptor is not their landmark's."""

    def __init__(self, L, n_land=20000, seed=17, shuffle=0.2, px=0.7, desc_noise=0.03, dropout=0.03, cap=400):
        self.L, self.fr = L, loop_frames(L)
        self.P, self.D = landmarks(self.fr, n_land=n_land, seed=seed)
        rng = np.random.default_rng(seed + 1)
        self.sal = rng.uniform(0.0, 1.0, len(self.P))
        self.seed, self.shuffle, self.px, self.dn, self.dropout, self.cap = seed, shuffle, px, desc_noise, dropout, cap

    def frame(self, g, key=None):
        """key: the noise draw (default g): a held camera re-observes rendered frame g with fresh noise."""
        U = len(self.fr)
        f = self.fr[g % U]
        rng = np.random.default_rng((self.seed, g if key is None else key))
        idx, u, v = visible(f, self.P)
        score = self.sal[idx] * (1.0 + rng.normal(0, 0.1, len(idx)))
        idx = idx[np.argsort(-score, kind="stable")[:self.cap]]
        n = len(idx)
        k = np.zeros(n, KP_DTYPE)
        k["x"] = u[idx] + rng.normal(0, self.px, n)
        k["y"] = v[idx] + rng.normal(0, self.px, n)
        k["size"], k["angle"], k["response"], k["class_id"] = 8.0, -1.0, 0.5, -1
        src = idx.copy()
        sel = np.nonzero(rng.random(n) < self.shuffle)[0]
        if len(sel) > 1:
            src[sel] = idx[np.roll(sel, 1 + int(rng.integers(0, len(sel) - 1)))]
        d = self.D[src] + rng.normal(0, self.dn, (n, 256)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        depth = self.L["depth"][g % U].copy()
        depth[rng.random(depth.shape) < self.dropout] = 0.0
        return k, d.astype(np.float32), depth, idx, src != idx
