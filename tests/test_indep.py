"""The independent numpy restatements (tests/indep.py, the producers of the fmat / emat / pnp / ba
golden values) against known answers and against the oracle on fresh seeded problems: identical
RANSAC decisions and masks, values within the golden tolerances (test_golden.py)."""
import numpy as np
import pytest

import indep


def _rot_angle(Ra, Rb):
    return float(np.arccos(np.clip((np.trace(Ra.T @ Rb) - 1) / 2, -1, 1)))


@pytest.mark.parametrize("n,seed,noise,out", [(40, 201, 0.0, 0.0), (150, 202, 0.6, 0.3)])
def test_pnp_independent_equals_oracle(oracle, n, seed, noise, out):
    from test_oracle_pnp import pnp_problem
    obj, img, R, t, outl = pnp_problem(n, seed, noise=noise, outlier_frac=out)
    ok, rv, tv, inl, mask, diag = indep.pnp_ransac(obj, img, 100)
    oo = oracle.pnp_ransac(obj, img, 100)
    assert ok and np.array_equal(oo[4].astype(bool), mask) and oo[3] == inl
    # the winning iteration is compared only without noise: on noisy 5-point subsets EPnP's choice
    # between its N = 4 / 2 / 3 approximations can turn on rounding when two reprojection errors
    # tie, so independent arithmetic may reach the same consensus set at another iteration
    if noise == 0.0:
        assert list(oo[5][:2]) == list(diag)
    s, Rw, tw, c = indep.solve_pnp(obj, img, 100, 10)
    so, Ro, to, co = oracle.solve_pnp(obj, img, 100, 10)
    assert s and so and c == co and np.max(np.abs(Rw - Ro)) < 1e-8 and np.max(np.abs(tw - to)) < 1e-8
    if noise == 0.0:
        assert _rot_angle(Rw, R.T) < 1e-6


@pytest.mark.parametrize("seed", [202, 5, 7])
def test_epnp_hypotheses_independent_equal_oracle(oracle, seed):
    """Every RANSAC hypothesis, not only the winner: EPnP on the cv::RNG 5-point subsets (and
    4-point problems) equals numpy's restatement to 1e-9.  This holds because both take the same
    basis of the subset's 2-dimensional null space (the QR basis of M^T from sign-canonical control
    points, pnp_solvers.h epnp_small_eig) -- the N = 2 / 3 approximations depend on that basis."""
    from test_oracle_pnp import pnp_problem, cv_rng
    obj, img, R, t, outl = pnp_problem(150, seed, noise=0.6, outlier_frac=0.3)
    g, n, worst, count = cv_rng(), len(obj), 0.0, 0
    for it in range(300):
        idx = []
        m = 4 if it % 10 == 9 else 5
        while len(idx) < m:
            v = next(g) % n
            if v not in idx:
                idx.append(v)
        ok, Ro, to = oracle.epnp(obj[idx].astype(np.float64), img[idx].astype(np.float64))
        r = indep.epnp(obj[idx], img[idx], (525.0, 525.0, 319.5, 239.5))
        assert bool(ok) == (r is not None)
        if r is None:
            continue
        count += 1
        worst = max(worst, np.abs(Ro - r[0]).max(), np.abs(to - r[1]).max() / max(1.0, np.abs(r[1]).max()))
    assert count > 250 and worst < 1e-9


@pytest.mark.parametrize("n,seed,noise,out", [(80, 203, 0.0, 0.0), (200, 204, 0.5, 0.35), (14, 205, 0.4, 0.0)])
def test_fundamental_independent_equals_oracle(oracle, n, seed, noise, out):
    from test_oracle_fmat import two_view
    p1, p2, F, outl = two_view(n, seed, noise, out)
    ok, Fi, mask, diag = indep.find_fundamental(p1, p2)
    oko, Fo, masko, diago = oracle.find_fundamental(p1, p2)
    assert ok and oko and list(diago) == list(diag) and np.array_equal(masko.astype(bool), mask)
    assert np.max(np.abs(Fo - Fi)) <= 1e-9 * np.abs(Fi).max()


@pytest.mark.parametrize("n,seed,noise,out", [(50, 206, 0.0, 0.0), (120, 207, 0.3, 0.25)])
def test_essential_independent_equals_oracle(oracle, n, seed, noise, out):
    from test_oracle_emat import two_view
    p1, p2, R, t, X, outl = two_view(n, seed, noise=noise, outlier_frac=out)
    ok, Ri, ti, mask, inl, good = indep.estimate_motion(p1, p2)
    oko, Ro, to, masko, inlo, goodo = oracle.estimate_motion(p1, p2)
    assert ok and oko and inl == inlo and good == goodo
    assert np.max(np.abs(Ro - Ri)) <= 1e-7 and np.max(np.abs(to - ti)) <= 1e-6
    if noise == 0.0:
        assert _rot_angle(Ri, R) < 1e-6


def test_five_point_known_answer():
    rng = np.random.default_rng(3)
    R = indep.rod_v2m(rng.normal(size=3) * 0.2)
    t = rng.normal(size=3)
    t /= np.linalg.norm(t)
    X = np.stack([rng.uniform(-1, 1, 5), rng.uniform(-1, 1, 5), rng.uniform(3, 6, 5)], 1)
    q1 = X[:, :2] / X[:, 2:]
    Y = X @ R.T + t
    q2 = Y[:, :2] / Y[:, 2:]
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    Et = tx @ R
    Et /= np.linalg.norm(Et)
    Es = indep.five_point(q1, q2)
    assert 1 <= len(Es) <= 10
    assert min(min(np.abs(E - Et).max(), np.abs(E + Et).max()) for E in Es) < 1e-8


def test_local_ba_independent_equals_oracle(oracle):
    from test_oracle_ba import ba_problem
    R, t, P, P0, kf, pt, uv = ba_problem(N=5, M=120, seed=208, noise=0.5, pert=0.04, outliers=3)
    Ri, ti, Pi, eb, ea, st = indep.local_ba(R, t, P0, kf, pt, uv)
    Ro, to, Po, ebo, eao, so = oracle.local_ba(R, t, P0, kf, pt, uv)
    assert list(so[:2]) == list(st) and ea < eb
    assert abs(ebo - eb) <= 1e-9 * eb and abs(eao - ea) <= 1e-9 * ea
    assert np.max(np.abs(Po - Pi)) <= 1e-9 and np.max(np.abs(Ro - Ri)) <= 1e-9 and np.max(np.abs(to - ti)) <= 1e-9
