"""The tracking loop's glue pinned independently.

The oracle tracker (host/tracker.hpp over the CPU stages; == the GPU tracker bit for bit, tests/
test_gpu_tracker_bench.py, test_tracker_noisy.py) writes an op log (VS_OPLOG, oracle/orc_slam.cpp): every
back-end call with the inputs its glue chose and the kernel outputs it got.  tests/slam_glue_ref.py —
Slam::process_frame (Slam.cpp:809-1135) restated in numpy from the reference and Config.h alone, sharing
no source with tracker.hpp — replays the log: for every frame it makes its own decisions on the logged
kernel outputs (bridge, recovery gate, 3D-3D vs E fallback, EKF predict / update / innovation gate / step
clamp, keyframe and proactive-keyframe rules, periodic PnP, triangulation, depth points, culling
cadence), checks the inputs of every call the C++ glue made against its own state (reference frame,
3D-3D seed, the pose of local-map tracking, the correspondences of every PnP, the projection matrices of
every triangulation, the visibility flags) and compares each frame's outcome: return value, keyframe
flag, pose (<= 1e-9), map size / valid points, frame and keyframe counts, match count."""
import os

import numpy as np
import pytest

import landmarks
import slam_glue_ref
import synth

T0 = 1311868164.0
U = 126


@pytest.fixture(scope="module")
def loop():
    return synth.loop_sequence(U, workers=8)


def _replay(oracle, frames, tmp_path, name, accel=None):
    log = str(tmp_path / f"{name}.jsonl")
    os.environ["VS_OPLOG"] = log
    try:
        S = oracle.Slam()
    finally:
        del os.environ["VS_OPLOG"]
    if accel is not None:  # main.cpp:1060-1066: initial pose, accelerometer stream, gravity direction
        S.set_initial_pose(np.eye(3), np.zeros(3))
        S.set_accelerometer(accel)
    for fid, ts, k, d, dep in frames:
        S.process(k, d, dep, ts, fid)
    stats = S.stats()
    edges, cons = S.loops()
    S.close()  # flushes and closes the log
    G = slam_glue_ref.GlueRef(log)
    if accel is not None:
        G.set_initial_pose(np.eye(3), np.zeros(3))
        G.set_accelerometer(accel)
    for fid, ts, k, d, dep in frames:
        G.process_frame(slam_glue_ref.Frame(fid, ts, k, dep))
    # loop closure: the edges and PGO constraints the restatement derived == the C++ glue's
    assert [tuple(e) for e in edges.tolist()] == G.loop_edges, (edges, G.loop_edges)
    assert len(cons) == len(G.loop_constraints)
    for c, (a, b, R, t, ts_, rs) in zip(cons, G.loop_constraints):
        assert (int(c[0]), int(c[1])) == (a, b) and c[14] == ts_ and c[15] == rs
        assert np.abs(c[2:11] - R.ravel()).max() < 1e-9 and np.abs(c[11:14] - t).max() < 1e-9
    # the C++ glue's decision counters (vs_slam_stats order) == the restatement's
    import vslam_abi
    st = dict(zip(vslam_abi.SLAM_STATS, stats.tolist()))
    for key in ("via_3d3d", "via_emat", "emat_failed", "bridges", "recoveries", "recovery_failed", "pnp_refined",
                "periodic_pnp", "triangulated", "depth_points", "culled"):
        assert st[key] == G.counts[key], (key, st[key], G.counts[key])
    assert st["keyframes"] == G.keyframe_count and st["map_points"] == len(G.mp_pos)
    assert st["map_valid"] == G._n_valid() and st["frame_count"] == G.frame_count
    assert st["stationary"] == G.counts["stationary"] and st["chains_recomputed"] == G.counts["chains_recomputed"]
    assert st["loop_count"] == G.loop_count
    return G, stats


def _noisy(loop, n, **kw):
    NS = landmarks.NoisySequence(loop, **kw)
    out = []
    for g in range(n):
        k, d, dep, _, _ = NS.frame(g)
        out.append((3 * g, T0 + 0.1 * g, k, d, dep))
    return out


def test_glue_restatement_replays_300_noisy_frames(oracle, loop, tmp_path):
    frames = _noisy(loop, 300, shuffle=0.35, desc_noise=0.015)
    G, stats = _replay(oracle, frames, tmp_path, "noisy")
    print(_branches(G), G.counts)
    assert len(G.frames) == 300 and G.counts["via_3d3d"] == 299 and G.counts["cull_rounds"] > 10


def _branches(G):
    return {k: sum(1 for b in G.branch.values() if b == k) for k in sorted(set(G.branch.values()))}


def test_glue_restatement_replays_a_monocular_stretch(oracle, loop, tmp_path):
    """No depth: every frame takes the E-matrix fallback with the scale fallback (Slam.cpp:965-984),
    keyframes triangulate by DLT alone and create no depth points."""
    frames = [(fid, ts, k, d, None) for fid, ts, k, d, _ in _noisy(loop, 160, shuffle=0.2, desc_noise=0.015)]
    G, stats = _replay(oracle, frames, tmp_path, "mono")
    br = _branches(G)
    print(br, G.counts)
    assert br.get("emat", 0) > 100 and G.counts["depth_points"] == 0


def test_glue_restatement_replays_a_perturbed_sequence(oracle, loop, tmp_path):
    """Frame drops, a stretch without depth, a frame with too few keypoints and jumps along the path:
    the bridge keyframe, PnP recovery, rejection and E-fallback branches of Slam.cpp:820-984."""
    NS = landmarks.NoisySequence(loop, shuffle=0.3, desc_noise=0.015)
    rng = np.random.default_rng(5)
    frames, g, fid = [], 0, 0
    while len(frames) < 260:
        k, d, dep, _, _ = NS.frame(g)
        n = len(frames)
        if 60 <= n < 70:
            dep = None                                  # depth dropouts: E-matrix fallback
        if n in (90, 150):
            keep = rng.permutation(len(k))[:20]         # too few keypoints: rejected
            k, d = k[keep], d[keep]
        if 120 <= n < 124 or 200 <= n < 203:
            keep = rng.permutation(len(k))[:60]         # few features: weak matches to the keyframe
            k, d = k[keep], d[keep]
        frames.append((fid, T0 + 0.1 * g, k, d, dep))
        step = 1 if n < 100 else (3 if n < 180 else 5)  # faster motion later on
        g += step
        fid += 3 * step
    G, stats = _replay(oracle, frames, tmp_path, "perturbed")
    br = _branches(G)
    print(br, G.counts)
    c = G.counts
    assert br.get("rejected", 0) >= 2 and br.get("emat", 0) >= 5 and c["bridges"] >= 1 and c["recovery_failed"] >= 1
    assert c["ekf_gated"] >= 1 and c["ekf_clamped"] >= 1 and c["proactive_kf"] >= 1 and c["periodic_pnp"] >= 1


def test_glue_restatement_replays_a_stop_with_an_accelerometer(oracle, loop, tmp_path):
    """The accelerometer branches: a drive that stops for 14 frames (the camera holds
    its pose; every held frame observes it with fresh noise) with a 100 Hz accelerometer stream whose
    vibration drops while held.  The restatement computes the gravity axis and the initial height
    itself (Slam.cpp:1587-1616), decides every frame's stationarity from the stream (:1621-1651),
    restates the stationary frame (:618-694: local-map tracking, the rotation-only PnP update, the
    0.25 rad keyframe rule, the EKF velocity reset), the post-stationary re-match / F / motion
    (:916-951) and the height update of every visual EKF step (:1013-1016, :1720-1744)."""
    NS = landmarks.NoisySequence(loop, shuffle=0.3, desc_noise=0.015)
    n1, hold, n2 = 30, 14, 40
    gs = list(range(n1)) + [n1 - 1] * hold + list(range(n1, n1 + n2))
    frames = []
    for k, g in enumerate(gs):
        kp, d, dep, _, _ = NS.frame(g, key=1000 + k)
        frames.append((3 * k, T0 + 0.1 * k, kp, d, dep))
    rng = np.random.default_rng(71)
    ta = np.arange(-0.5, 0.1 * len(gs) + 0.5, 0.01)
    held = (ta >= 0.1 * n1 - 0.05) & (ta <= 0.1 * (n1 + hold - 1) + 0.05)
    sd = np.where(held, 0.02, 0.6)
    acc = np.stack([T0 + ta, rng.standard_normal(ta.size) * sd, -9.81 + rng.standard_normal(ta.size) * sd,
                    rng.standard_normal(ta.size) * sd], axis=1)
    G, stats = _replay(oracle, frames, tmp_path, "stationary", accel=acc)
    br = _branches(G)
    print(br, G.counts, G.gravity, G.initial_height)
    assert br.get("stationary", 0) >= hold - 2 and G.counts["chains_recomputed"] >= 1
    assert G.gravity is not None and np.count_nonzero(G.gravity) == 1 and G.has_initial_height


def test_glue_restatement_replays_loop_closures(oracle, loop, tmp_path):
    """Loop closure: 420 frames at four rendered frames per processed frame make every
    frame a keyframe, so LoopCloser::detect runs at keyframes 200 and 400 (Slam.cpp:1084-1086) with
    the drive on its third and fourth lap.  The restatement picks the candidates (every 5th keyframe
    at least 200 ids back, LoopCloser.cpp:44-49) and the best one from the logged per-candidate match
    and E-RANSAC inlier counts, gathers the map points observed near it, checks the FLANN input, and
    applies the PnP verification and jump gates; its loop edges and PGO constraints equal the glue's."""
    NS = landmarks.NoisySequence(loop, shuffle=0.3, desc_noise=0.015)
    frames = []
    for k in range(420):
        kp, d, dep, _, _ = NS.frame(4 * k)
        frames.append((12 * k, T0 + 0.4 * k, kp, d, dep))
    G, stats = _replay(oracle, frames, tmp_path, "loops")
    print(_branches(G), G.counts, G.loop_edges)
    assert G.keyframe_count >= 400 and G.counts["loops_detected"] >= 2 and G.counts["loop_constraints"] >= 1
