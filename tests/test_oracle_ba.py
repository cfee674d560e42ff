"""CPU tests pinning the local bundle adjustment restatement (A14, reference
src/Optimizer.cpp:187-599).

* one LM step equals an independent numpy solve of the full (unreduced) damped normal equations
  built from the same Jacobian definitions — the Schur complement, per-point inverses and
  back-substitution must reproduce it;
* known answer: noise-free observations with perturbed points converge to the true structure while
  the 1e10 pose damping keeps the poses (structure-only in practice);
* the reference's bail-outs."""
import numpy as np
import pytest

import restate

K = (525.0, 525.0, 319.5, 239.5)


def ba_problem(N=5, M=120, seed=0, noise=0.0, pert=0.05, outliers=0):
    rng = np.random.default_rng(seed)
    Rs, ts = [], []
    for i in range(N):  # camera -> world poses along a short arc
        Rs.append(restate.rodrigues(np.array([0.0, 0.04 * i, 0.01 * i])))
        ts.append(np.array([0.15 * i, 0.02 * i, 0.0]))
    P = np.stack([rng.uniform(-2, 2.5, M), rng.uniform(-1.5, 1.5, M), rng.uniform(3.0, 7.0, M)], 1)
    kf, pt, uv = [], [], []
    for i in range(N):  # keyframe-major gather order (Optimizer.cpp:224-243), shuffled keypoint order
        pc = (P - ts[i]) @ Rs[i]
        u = K[0] * pc[:, 0] / pc[:, 2] + K[2]
        v = K[1] * pc[:, 1] / pc[:, 2] + K[3]
        vis = np.flatnonzero((pc[:, 2] > 0.1) & (u > 0) & (u < 640) & (v > 0) & (v < 480) &
                             (rng.uniform(size=M) < 0.85))
        for j in rng.permutation(vis):
            kf.append(i)
            pt.append(j)
            uv.append([u[j] + rng.normal() * noise, v[j] + rng.normal() * noise])
    uv = np.array(uv)
    if outliers:
        idx = rng.choice(len(uv), outliers, replace=False)
        uv[idx] += 40.0
    P0 = P + rng.normal(size=P.shape) * pert
    return np.array(Rs), np.array(ts), P, P0, np.array(kf, np.int32), np.array(pt, np.int32), uv


def _jac(rv, t, P, u_obs, v_obs):
    """The reference's per-observation Jacobian rows (Optimizer.cpp:331-405), weighted by sqrt(w)."""
    fx, fy, cx, cy = K
    R = restate.rodrigues(rv)
    d = P - t
    X, Y, Z = R.T @ d
    u, v = fx * X / Z + cx, fy * Y / Z + cy
    ru, rvv = u - u_obs, v - v_obs
    rn = np.hypot(ru, rvv)
    w = 5.0 / rn if rn > 5.0 else 1.0
    sw = np.sqrt(w)
    D = np.array([[fx / Z, 0, -fx * X / Z ** 2], [0, fy / Z, -fy * Y / Z ** 2]])
    Jm = D @ R.T * sw
    Jr = np.zeros((2, 3))
    for k in range(3):
        rp = rv.copy()
        rp[k] += 1e-6
        Xp, Yp, Zp = restate.rodrigues(rp).T @ d
        Jr[:, k] = [(fx * Xp / Zp + cx - u) / 1e-6 * sw, (fy * Yp / Zp + cy - v) / 1e-6 * sw]
    return np.hstack([Jr, -Jm]), Jm, np.array([ru, rvv]) * sw


def test_one_step_equals_full_normal_equations(oracle):
    R, t, P, P0, kf, pt, uv = ba_problem(N=4, M=60, seed=1, noise=0.3, pert=0.02, outliers=3)
    N, M = len(R), len(P)
    rv = np.array([oracle.rodrigues(r) for r in R])
    n = 6 * N + 3 * M
    H = np.zeros((n, n))
    g = np.zeros(n)
    for o in range(len(kf)):
        i, j = kf[o], pt[o]
        Jp, Jm, r = _jac(rv[i], t[i], P0[j], uv[o, 0], uv[o, 1])
        J = np.zeros((2, n))
        J[:, 6 * i:6 * i + 6] = Jp
        J[:, 6 * N + 3 * j:6 * N + 3 * j + 3] = Jm
        H += J.T @ J
        g += J.T @ r
    lam = 1e-4
    for i in range(N):
        H[6 * i:6 * i + 6, 6 * i:6 * i + 6] += 1e10 * np.eye(6)
    H[np.diag_indices(n)] *= 1 + lam
    delta = np.linalg.solve(H, -g)
    R1, t1, P1, eb, ea, st = oracle.local_ba(R, t, P0, kf, pt, uv, max_iter=1)
    assert st[0] == 1 and st[1] == 1  # the first step is accepted on this problem
    dm = (P1 - P0).ravel()
    want = delta[6 * N:]
    assert np.max(np.abs(dm - want)) <= 1e-7 * np.max(np.abs(want))
    # poses 1..N-1 move by the (tiny, 1e10-damped) pose step
    assert np.max(np.abs(t1[1:] - (t[1:] + delta[:6 * N].reshape(N, 6)[1:, 3:]))) < 1e-12
    assert np.array_equal(t1[0], t[0])


def test_known_answer_structure_converges(oracle):
    R, t, P, P0, kf, pt, uv = ba_problem(N=6, M=150, seed=2)
    R1, t1, P1, eb, ea, st = oracle.local_ba(R, t, P0, kf, pt, uv)
    assert st[2] == 1 and eb > 1.0 and ea < 1e-3 * eb
    seen = np.unique(pt)
    multi = [j for j in seen if len(np.unique(kf[pt == j])) >= 2]
    assert np.max(np.abs(P1[multi] - P[multi])) < 1e-3
    assert np.max(np.abs(t1 - t)) < 1e-6 and np.max(np.abs(R1 - R)) < 1e-6


def test_bailouts(oracle):
    R, t, P, P0, kf, pt, uv = ba_problem(N=3, M=50, seed=3)
    assert oracle.local_ba(R[:1], t[:1], P0, kf[kf == 0], pt[kf == 0], uv[kf == 0])[5][2] == 0  # N < 2
    assert oracle.local_ba(R, t, P0, kf[:19], pt[:19], uv[:19])[5][2] == 0                     # obs < 20
    keep = pt < 9
    assert oracle.local_ba(R, t, P0[:9], kf[keep], pt[keep], uv[keep])[5][2] == 0              # M < 10
    R1, t1, P1, eb, ea, st = oracle.local_ba(R, t, P0, kf[:19], pt[:19], uv[:19])
    assert eb == ea == 0 and np.array_equal(P1, P0)
