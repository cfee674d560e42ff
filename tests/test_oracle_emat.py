"""CPU tests pinning the essential-matrix path restatement (A12: Slam::estimate_motion, reference
src/Slam.cpp:1193-1213, and the depth scale estimators :73-207).

OpenCV's findEssentialMat / recoverPose are absent, so parity with OpenCV is unpinned; the oracle is
pinned by known answers (noise-free two-view geometry: the 5-point solutions contain the true E,
recoverPose returns the true R and the direction of t), an independent Python replay of the RANSAC
driver (cv::RNG subsets, Sampson errors in numpy), and a literal numpy restatement of the scale
estimators (exact equality)."""
import math

import numpy as np
import pytest

import restate
from test_oracle_pnp import cv_rng, ransac_update_num_iters

K = (525.0, 525.0, 319.5, 239.5)


def skew(t):
    return np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])


def two_view(n, seed, R=None, t=None, noise=0.0, outlier_frac=0.0):
    """Camera 1 = [I|0], camera 2: x2 = R x1 + t.  Returns pixel pts (f32), R, t, depth1 and labels."""
    rng = np.random.default_rng(seed)
    R = restate.rodrigues(rng.normal(size=3) * 0.05) if R is None else R
    t = np.array([0.2, 0.03, 0.05]) + rng.normal(size=3) * 0.02 if t is None else t
    X = np.stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(2, 8, n)], 1)
    X2 = X @ R.T + t
    p1 = np.stack([K[0] * X[:, 0] / X[:, 2] + K[2], K[1] * X[:, 1] / X[:, 2] + K[3]], 1)
    p2 = np.stack([K[0] * X2[:, 0] / X2[:, 2] + K[2], K[1] * X2[:, 1] / X2[:, 2] + K[3]], 1)
    p1 = p1 + rng.normal(size=p1.shape) * noise
    p2 = p2 + rng.normal(size=p2.shape) * noise
    out = np.zeros(n, bool)
    m = int(round(outlier_frac * n))
    if m:
        idx = rng.choice(n, m, replace=False)
        out[idx] = True
        p2[idx] = np.stack([rng.uniform(0, 640, m), rng.uniform(0, 480, m)], 1)
    return p1.astype(np.float32), p2.astype(np.float32), R, t, X, out


def norm_q(p):
    p = np.asarray(p, np.float64)
    return np.stack([(p[:, 0] - K[2]) / K[0], (p[:, 1] - K[3]) / K[1]], 1)


def e_close(Ea, Eb, tol):
    a = Ea / np.linalg.norm(Ea)
    b = Eb / np.linalg.norm(Eb)
    return min(np.max(np.abs(a - b)), np.max(np.abs(a + b))) < tol


@pytest.mark.parametrize("case", ["generic", "sideways_R_identity", "forward"])
def test_five_point_known_answer(oracle, case):
    rng = np.random.default_rng(["generic", "sideways_R_identity", "forward"].index(case) + 11)
    if case == "generic":
        R, t = restate.rodrigues(rng.normal(size=3) * 0.2), rng.normal(size=3)
    elif case == "sideways_R_identity":  # e33 = 0: not representable with a fixed E3 coefficient basis
        R, t = np.eye(3), np.array([1.0, 0.0, 0.0])
    else:
        R, t = restate.rodrigues(np.array([0.0, 0.1, 0.0])), np.array([0.0, 0.1, 1.0])
    X = np.stack([rng.uniform(-2, 2, 5), rng.uniform(-2, 2, 5), rng.uniform(3, 6, 5)], 1)
    X2 = X @ R.T + t
    q1, q2 = X[:, :2] / X[:, 2:], X2[:, :2] / X2[:, 2:]
    Es = oracle.five_point(q1, q2)
    assert 1 <= len(Es) <= 10
    Et = skew(t) @ R
    assert any(e_close(E, Et, 1e-7) for E in Es)
    for E in Es:  # every returned solution is an essential matrix through the 5 points
        assert abs(np.linalg.det(E)) < 1e-9
        assert np.max(np.abs(2 * E @ E.T @ E - np.trace(E @ E.T) * E)) < 1e-9
        h1, h2 = np.c_[q1, np.ones(5)], np.c_[q2, np.ones(5)]
        assert np.max(np.abs(np.sum(h2 * (h1 @ E.T), 1))) < 1e-9


def test_five_point_accuracy_sweep(oracle):
    """300 random minimal problems: the true E is recovered to 1e-7 in >= 97% of them (the rest
    are near-double roots of the degree-10 polynomial, still within 1e-3)."""
    errs = []
    for s in range(300):
        rng = np.random.default_rng(s)
        R, t = restate.rodrigues(rng.normal(size=3) * 0.2), rng.normal(size=3)
        X = np.stack([rng.uniform(-2, 2, 5), rng.uniform(-2, 2, 5), rng.uniform(3, 6, 5)], 1)
        X2 = X @ R.T + t
        Es = oracle.five_point(X[:, :2] / X[:, 2:], X2[:, :2] / X2[:, 2:])
        Et = skew(t) @ R
        errs.append(min(next((tol for tol in (1e-7, 1e-3) if e_close(E, Et, tol)), 1.0) for E in Es))
    errs = np.array(errs)
    assert np.mean(errs <= 1e-7) >= 0.97 and np.all(errs <= 1e-3)


def sampson(E, q1, q2):
    h1, h2 = np.c_[q1, np.ones(len(q1))], np.c_[q2, np.ones(len(q2))]
    Ex1, Etx2 = h1 @ E.T, h2 @ E
    r = np.sum(h2 * Ex1, 1)
    return (r * r / (Ex1[:, 0] ** 2 + Ex1[:, 1] ** 2 + Etx2[:, 0] ** 2 + Etx2[:, 1] ** 2)).astype(np.float32)


def replay(oracle, p1, p2, prob=0.999, thr_px=1.0, max_iters=1000):
    q1, q2 = norm_q(p1), norm_q(p2)
    n = len(q1)
    thr2 = np.float32((thr_px / ((K[0] + K[1]) / 2)) ** 2)
    g = cv_rng()
    niters, best, best_iter, bestE, it = max_iters, 0, -1, None, 0
    while it < niters:
        idx = []
        while len(idx) < 5:
            v = next(g) % n
            if v not in idx:
                idx.append(v)
        for E in oracle.five_point(q1[idx], q2[idx]):
            cnt = int((sampson(E, q1, q2) <= thr2).sum())
            if cnt > max(best, 4):
                best, best_iter, bestE = cnt, it, E
                niters = ransac_update_num_iters(prob, (n - cnt) / n, 5, niters)
        it += 1
    return it, best_iter, best, bestE


@pytest.mark.parametrize("n,seed,noise,out", [(80, 0, 0.3, 0.2), (200, 1, 0.5, 0.4), (40, 2, 0.2, 0.0)])
def test_find_essential_matches_replay(oracle, n, seed, noise, out):
    p1, p2, R, t, X, outl = two_view(n, seed, noise=noise, outlier_frac=out)
    ok, E, mask, diag = oracle.find_essential(p1, p2)
    it, best_iter, best, bestE = replay(oracle, p1, p2)
    assert ok and diag[0] == it and diag[1] == best_iter and diag[2] == best
    assert np.max(np.abs(E - bestE)) < 1e-12
    assert np.array_equal(mask, sampson(E, norm_q(p1), norm_q(p2)) <= np.float32((1.0 / 525.0) ** 2))


def test_find_essential_and_recover_pose_known_answer(oracle):
    p1, p2, R, t, X, outl = two_view(150, 3, outlier_frac=0.3)
    ok, E, mask, diag = oracle.find_essential(p1, p2)
    assert ok and not mask[outl].any() and mask[~outl].sum() >= (~outl).sum() - 2
    good, Rr, tr, m = oracle.recover_pose(E, p1, p2, mask.astype(np.uint8))
    assert good == m.sum() and good >= mask.sum() - 2
    assert np.max(np.abs(Rr - R)) < 1e-4
    assert np.max(np.abs(tr - t / np.linalg.norm(t))) < 1e-3


def test_estimate_motion_wrapper(oracle):
    p1, p2, R, t, X, outl = two_view(100, 4, noise=0.2, outlier_frac=0.1)
    ok, Rr, tr, mask, inl, good = oracle.estimate_motion(p1, p2)
    assert ok and inl >= 15 and good >= 15 and abs(np.linalg.det(Rr) - 1) < 0.01
    assert math.acos(min(1, (np.trace(Rr.T @ R) - 1) / 2)) < 2e-3
    assert not oracle.estimate_motion(p1[:4], p2[:4])[0]              # fewer than 5 points (:1195)
    rng = np.random.default_rng(0)
    q = np.stack([rng.uniform(0, 640, 30), rng.uniform(0, 480, 30)], 1).astype(np.float32)
    assert not oracle.estimate_motion(q, q[::-1].copy())[0]            # no consistent motion


def scale_restated(p1, p2, R, t, d1, d2):
    """Literal numpy restatement of Slam::estimate_scale_from_depth / _single_depth."""
    fx, fy, cx, cy = K
    rnd = lambda v: int(math.floor(abs(v) + 0.5)) * (1 if v >= 0 else -1)  # noqa: E731  std::round
    h, w = d1.shape

    def single():
        sc = []
        for (x1, y1), (x2, y2) in zip(p1, p2):
            px, py = rnd(float(x1)), rnd(float(y1))
            if not (0 <= px < w and 0 <= py < h):
                continue
            z = d1[py, px]
            if z <= np.float32(0.1) or z > np.float32(10.0):
                continue
            z = float(z)
            P1 = [(float(x1) - cx) * z / fx, (float(y1) - cy) * z / fy, z]
            Rp = [R[r, 0] * P1[0] + R[r, 1] * P1[1] + R[r, 2] * P1[2] for r in range(3)]
            a = (float(x2) - cx) / fx
            if abs(t[0] - a * t[2]) > 1e-4:
                s = (a * Rp[2] - Rp[0]) / (t[0] - a * t[2])
                if 0.001 < s < 100.0:
                    sc.append(s)
            b = (float(y2) - cy) / fy
            if abs(t[1] - b * t[2]) > 1e-4:
                s = (b * Rp[2] - Rp[1]) / (t[1] - b * t[2])
                if 0.001 < s < 100.0:
                    sc.append(s)
        return sorted(sc)[len(sc) // 2] if len(sc) >= 10 else -1.0

    if d2 is None:
        return single()
    sc = []
    for (x1, y1), (x2, y2) in zip(p1, p2):
        px1, py1, px2, py2 = rnd(float(x1)), rnd(float(y1)), rnd(float(x2)), rnd(float(y2))
        if not (0 <= px1 < w and 0 <= py1 < h and 0 <= px2 < w and 0 <= py2 < h):
            continue
        z1, z2 = d1[py1, px1], d2[py2, px2]
        if z1 <= np.float32(0.1) or z1 > np.float32(10.0) or z2 <= np.float32(0.1) or z2 > np.float32(10.0):
            continue
        z1, z2 = float(z1), float(z2)
        P1 = [(float(x1) - cx) * z1 / fx, (float(y1) - cy) * z1 / fy, z1]
        P2 = [(float(x2) - cx) * z2 / fx, (float(y2) - cy) * z2 / fy, z2]
        d = [P2[r] - (R[r, 0] * P1[0] + R[r, 1] * P1[1] + R[r, 2] * P1[2]) for r in range(3)]
        s = d[0] * t[0] + d[1] * t[1] + d[2] * t[2]  # scalar order of the reference's expression
        if 0.001 < s < 50.0:
            sc.append(s)
    if len(sc) < 10:
        return single()
    sc.sort()
    q1, q3 = sc[len(sc) // 4], sc[3 * len(sc) // 4]
    lo, hi = q1 - 1.5 * (q3 - q1), q3 + 1.5 * (q3 - q1)
    f = sorted(s for s in sc if lo <= s <= hi)
    return f[len(f) // 2] if f else sc[len(sc) // 2]


def _depth_maps(X, R, t, p1, p2):
    d1 = np.zeros((480, 640), np.float32)
    d2 = np.zeros((480, 640), np.float32)
    X2 = X @ R.T + t
    for i in range(len(X)):
        x1, y1 = int(round(float(p1[i, 0]))), int(round(float(p1[i, 1])))
        x2, y2 = int(round(float(p2[i, 0]))), int(round(float(p2[i, 1])))
        if 0 <= x1 < 640 and 0 <= y1 < 480:
            d1[y1, x1] = X[i, 2]
        if 0 <= x2 < 640 and 0 <= y2 < 480:
            d2[y2, x2] = X2[i, 2]
    return d1, d2


def test_estimate_scale_known_answer_and_restatement(oracle):
    p1, p2, R, t, X, outl = two_view(150, 5)
    s_true = np.linalg.norm(t)
    t_unit = t / s_true
    d1, d2 = _depth_maps(X, R, t, p1, p2)
    s2 = oracle.estimate_scale(p1, p2, R, t_unit, d1, d2)
    s1 = oracle.estimate_scale(p1, p2, R, t_unit, d1, None)
    assert s2 == scale_restated(p1, p2, R, t_unit, d1, d2)
    assert s1 == scale_restated(p1, p2, R, t_unit, d1, None)
    assert abs(s2 - s_true) < 0.02 * s_true and abs(s1 - s_true) < 0.02 * s_true
    # too few depth samples -> -1 (Slam.cpp:190)
    assert oracle.estimate_scale(p1[:5], p2[:5], R, t_unit, d1, None) == -1.0


def _found(roots, r, tol):
    return np.any(np.abs(roots - r) <= tol * max(1.0, abs(r)))


@pytest.mark.parametrize("seed", range(20))
def test_poly_real_roots_simple_roots(oracle, seed):
    """five_point's degree-10 real-root search (emat_solvers.h poly_real_roots) on polynomials with
    well separated real roots and complex pairs: every real root to 1e-12, none invented."""
    rng = np.random.default_rng(seed)
    nr = int(rng.integers(0, 6))
    real = np.sort(rng.uniform(-3, 3, nr))
    while nr > 1 and np.min(np.diff(real)) < 0.05:
        real = np.sort(rng.uniform(-3, 3, nr))
    poly = np.poly1d([1.0])
    for r in real:
        poly *= np.poly1d([1.0, -r])
    for _ in range((10 - nr) // 2):
        a, b = rng.uniform(-2, 2), rng.uniform(0.3, 2)
        poly *= np.poly1d([1.0, -2 * a, a * a + b * b])
    got = oracle.poly_real_roots(poly.coeffs[::-1] * rng.uniform(0.5, 2))
    assert len(got) == nr, (got, real)
    assert np.all(np.abs(got - real) <= 1e-12 * np.maximum(1, np.abs(real)))


@pytest.mark.parametrize("gap", [0.0, 1e-13, 1e-10, 1e-9, 1e-8])
def test_poly_real_roots_near_double_root(oracle, gap):
    """the derivative's roots (the cuts between monotone pieces) are refined to 2^-26 only,
    so a cut can land outside a pair of roots closer than that; the pair then shows no sign change on
    either side.  A cut at which the polynomial is within rounding noise of zero is taken as a root: a
    (near-)double root is never lost, and the separated roots stay exact."""
    poly = np.poly1d([1.0, -1.0]) * np.poly1d([1.0, -(1.0 + gap)])
    for r in (-2.5, 0.3, 2.0):
        poly *= np.poly1d([1.0, -r])
    poly *= np.poly1d([1.0, 0.4, 1.3]) * np.poly1d([1.0, -1.0, 2.0]) * np.poly1d([1.0, 3.0])
    got = oracle.poly_real_roots(poly.coeffs[::-1])
    assert 1 <= np.sum(np.abs(got - 1.0) < 1e-6) <= 2, got
    for r in (-3.0, -2.5, 0.3, 2.0):
        assert _found(got, r, 1e-12), (r, got)
    assert len(got) <= 7


def test_poly_real_roots_huge_root_bound(oracle):
    """A tiny leading coefficient puts the Cauchy bound near 1e280.  The search is capped where every
    derivative level's Horner sums stay finite (2^97 here: the root near -1e40 is not searched), the
    geometric bracket split takes sqrt|a| sqrt|b| (sqrt(a b) would overflow) and a bracket straddling 0
    that wide is split at 0 first, so the small roots come out exact instead of being lost to the
    iteration limit."""
    small = np.poly1d([1.0, -1.0]) * np.poly1d([1.0, -2.0]) * np.poly1d([1.0, -3.0])
    for lead in (1e-280, 1e-200, 1e-120):
        c = np.zeros(11)
        c[:4] = small.coeffs[::-1]
        c[10] = lead
        got = oracle.poly_real_roots(c)
        assert np.all(np.isfinite(got)) and np.all(np.abs(got) <= 2.0 ** 97), got
        for r in (1.0, 2.0, 3.0):
            assert _found(got, r, 1e-12), (lead, got)
        big = -(1.0 / lead) ** (1.0 / 7.0)  # x^7 ~ -c3 / c10 far out
        if abs(big) < 2.0 ** 90:
            assert _found(got, big, 1e-9), (big, got)
