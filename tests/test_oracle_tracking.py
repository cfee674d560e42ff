"""CPU tests pinning the oracle's track_local_map (A11), project_point (A15) and optimize_pose
(A13) against independent restatements and known answers."""
import numpy as np
import pytest

import restate


def _kps(oracle, kxy):
    k = np.zeros(len(kxy), oracle.KEYPOINT_DTYPE)
    k["x"], k["y"], k["size"], k["angle"], k["class_id"] = kxy[:, 0], kxy[:, 1], 8.0, -1.0, -1
    return k


@pytest.mark.parametrize("seed,n_kp,n_mp", [(0, 120, 400), (1, 400, 900), (2, 37, 300)])
def test_track_local_map_oracle_vs_python(oracle, seed, n_kp, n_mp):
    kxy, desc, pos, mdesc, valid, R, t = restate.synthetic_tracking_problem(n_kp, n_mp, seed)
    tr_o, kpmp_o, omp, okp = oracle.track_local_map(pos, mdesc, valid, _kps(oracle, kxy), desc, R, t)
    tr_p, kpmp_p, obs_p = restate.track_local_map_py(pos, mdesc, valid, kxy, desc, R, t)
    assert tr_o == tr_p > 0
    assert list(kpmp_o) == kpmp_p
    assert list(zip(omp.tolist(), okp.tolist())) == obs_p


def test_track_local_map_keeps_prior_assignments(oracle):
    kxy, desc, pos, mdesc, valid, R, t = restate.synthetic_tracking_problem(50, 10, 5)
    prior = np.arange(50, dtype=np.int32) + 1000
    tr, kpmp, _, _ = oracle.track_local_map(pos, mdesc, valid, _kps(oracle, kxy), desc, R, t, kp_to_mp=prior)
    changed = kpmp != prior
    assert changed.sum() <= tr and (kpmp[~changed] == prior[~changed]).all()


def test_rodrigues_matches_scipy(oracle):
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(0)
    for s in (1e-9, 1e-3, 0.5, 2.0, 3.1):  # rotation angles below pi (the vector is unique there)
        r = rng.normal(size=3)
        r *= s / np.linalg.norm(r)
        R = oracle.rodrigues(r)
        assert np.allclose(R, Rotation.from_rotvec(r).as_matrix(), atol=1e-14)
        assert np.allclose(oracle.rodrigues(R), r, atol=1e-9)
    # the theta ~ pi branch (s < 1e-5, c < 0)
    r = np.array([0.0, np.pi, 0.0])
    assert np.allclose(np.abs(oracle.rodrigues(oracle.rodrigues(r))), np.abs(r), atol=1e-7)


def test_project_point(oracle):
    R = restate.rodrigues(np.array([0.1, -0.2, 0.05]))
    t = np.array([0.3, -0.1, 0.2])
    pw = R @ np.array([0.2, -0.1, 2.0]) + t
    uv = oracle.project_point(pw, R, t)
    assert np.allclose(uv, [525 * 0.1 + 319.5, 525 * -0.05 + 239.5], atol=1e-12)
    assert list(oracle.project_point(R @ np.array([0, 0, -1.0]) + t, R, t)) == [-1.0, -1.0]


def pose_problem(n, seed, noise=0.0, perturb=(0.02, 0.03)):
    rng = np.random.default_rng(seed)
    R = restate.rodrigues(rng.normal(size=3) * 0.5)
    t = rng.normal(size=3)
    pc = np.stack([rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n), rng.uniform(1.0, 6.0, n)], 1)
    P = pc @ R.T + t
    uv = np.stack([525 * pc[:, 0] / pc[:, 2] + 319.5, 525 * pc[:, 1] / pc[:, 2] + 239.5], 1)
    uv = (uv + rng.normal(size=uv.shape) * noise).astype(np.float32)
    R0 = restate.rodrigues(rng.normal(size=3) * perturb[0]) @ R
    t0 = t + rng.normal(size=3) * perturb[1]
    return P, uv, R, t, R0, t0


@pytest.mark.parametrize("seed", [0, 1])
def test_optimize_pose_known_answer(oracle, seed):
    P, uv, R, t, R0, t0 = pose_problem(150, seed)
    Ro, to, eb, ea, stats = oracle.optimize_pose(P, uv, R0, t0)
    assert eb > 1.0 and ea < 1e-3 and ea < eb
    assert np.max(np.abs(Ro - R)) < 1e-5 and np.max(np.abs(to - t)) < 1e-5


def test_optimize_pose_too_few_points(oracle):
    P, uv, R, t, R0, t0 = pose_problem(2, 3)
    Ro, to, eb, ea, _ = oracle.optimize_pose(P, uv, R0, t0)
    assert eb == ea == 0 and np.array_equal(Ro, R0) and np.array_equal(to, t0)
