"""GPU parity for track_local_map (A11, bit-exact) and optimize_pose (A13, fp64 tolerance)."""
import numpy as np
import pytest

import restate
from test_oracle_tracking import _kps, pose_problem

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,n_kp,n_mp", [(0, 120, 400), (1, 400, 900), (2, 400, 20000), (3, 5, 3000), (4, 1024, 60000),
                                          (5, 1000, 12000)])
def test_track_local_map_bit_exact(vsctx, oracle, seed, n_kp, n_mp):
    kxy, desc, pos, mdesc, valid, R, t = restate.synthetic_tracking_problem(n_kp, n_mp, seed)
    kps = _kps(oracle, kxy)
    g = vsctx.track_local_map(pos, mdesc, valid, kps, desc, R, t)
    o = oracle.track_local_map(pos, mdesc, valid, kps, desc, R, t)
    assert g[0] == o[0] > 0
    assert np.array_equal(g[1], o[1])
    assert np.array_equal(g[2], o[2]) and np.array_equal(g[3], o[3])


def test_track_local_map_edges(vsctx, oracle):
    kxy, desc, pos, mdesc, valid, R, t = restate.synthetic_tracking_problem(30, 200, 7)
    kps = _kps(oracle, kxy)
    prior = np.arange(30, dtype=np.int32) + 500
    g = vsctx.track_local_map(pos, mdesc, valid, kps, desc, R, t, kp_to_mp=prior)
    o = oracle.track_local_map(pos, mdesc, valid, kps, desc, R, t, kp_to_mp=prior)
    assert g[0] == o[0] and np.array_equal(g[1], o[1])
    g = vsctx.track_local_map(pos[:0], mdesc[:0], valid[:0], kps, desc, R, t)  # empty map
    assert g[0] == 0 and (g[1] == -1).all()
    g = vsctx.track_local_map(pos, mdesc, valid, kps[:0], desc[:0], R, t)     # no keypoints
    assert g[0] == 0
    # observation capacity smaller than the number of observations
    g = vsctx.track_local_map(pos, mdesc, valid, kps, desc, R, t, obs_cap=3)
    assert g[0] == o[0] and len(g[2]) == 3 and np.array_equal(g[2], o[2][:3])


def test_track_local_map_on_pipeline_features(vsctx, oracle, seq4):
    # map = frame 0's keypoints back-projected with its depth (create_points_from_depth style),
    # tracked into frame 1 at its ground-truth pose
    feats = vsctx.extract_batch([f["bgr"] for f in seq4[:2]])
    (k0, d0), (k1, d1) = feats
    f0, f1 = seq4[0], seq4[1]
    pos, md = [], []
    for i in range(len(k0)):
        z = f0["depth"][int(k0["y"][i]), int(k0["x"][i])]
        if z <= 0.1:
            continue
        pc = np.array([(k0["x"][i] - 319.5) * z / 525.0, (k0["y"][i] - 239.5) * z / 525.0, z])
        pos.append(f0["R_wc"] @ pc + f0["t_wc"])
        md.append(d0[i])
    pos, md = np.array(pos), np.array(md, np.float32)
    valid = np.ones(len(pos), np.uint8)
    g = vsctx.track_local_map(pos, md, valid, k1, d1, f1["R_wc"], f1["t_wc"])
    o = oracle.track_local_map(pos, md, valid, k1, d1, f1["R_wc"], f1["t_wc"])
    assert g[0] == o[0] and np.array_equal(g[1], o[1]) and np.array_equal(g[2], o[2])


@pytest.mark.parametrize("seed,n,noise", [(0, 150, 0.0), (1, 400, 0.5), (2, 3, 0.0), (3, 2000, 1.0)])
def test_optimize_pose_matches_oracle(vsctx, oracle, seed, n, noise):
    P, uv, R, t, R0, t0 = pose_problem(n, seed, noise=noise)
    Rg, tg, ebg, eag = vsctx.optimize_pose(P, uv, R0, t0)
    Ro, to, ebo, eao, _ = oracle.optimize_pose(P, uv, R0, t0)
    # block-tree vs sequential sums: rounding-level differences only
    assert abs(ebg - ebo) <= 1e-9 * max(1.0, ebo)
    assert abs(eag - eao) <= 1e-6 * max(1.0, eao)
    assert np.max(np.abs(Rg - Ro)) <= 1e-8 and np.max(np.abs(tg - to)) <= 1e-8
    if noise == 0.0:
        assert eag < 1e-3


def test_optimize_pose_too_few_points(vsctx):
    P, uv, R, t, R0, t0 = pose_problem(2, 9)
    Rg, tg, eb, ea = vsctx.optimize_pose(P, uv, R0, t0)
    assert eb == ea == 0 and np.array_equal(Rg, R0) and np.array_equal(tg, t0)
