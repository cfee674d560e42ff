"""CPU tests pinning the F-matrix verification restatement (A8: reference src/Slam.cpp:880-910,
1174-1187, 1217-1240 over cv::findFundamentalMat(FM_RANSAC, 3.0, 0.999)).

OpenCV is absent and the reference ships no fixtures, so parity with OpenCV is unpinned; the
oracle is pinned by known answers (noise-free two-view scenes give F proportional to
K^-T [t]x R K^-1 and the ground-truth inlier mask) and by an independent numpy replay of the
registrators (cv::RNG subset stream with the collinearity rejection, 7-point solutions from a
numpy SVD null space and np.roots, the RANSAC / LMedS acceptance rules)."""
import math

import numpy as np
import pytest

import restate
from test_oracle_pnp import cv_rng, ransac_update_num_iters

K = np.array([[525.0, 0, 319.5], [0, 525.0, 239.5], [0, 0, 1]])


def two_view(n, seed, noise=0.0, outlier_frac=0.0):
    """pts1/pts2 (f32) of n points seen from two cameras; returns F_true (F(3,3)=1) and labels."""
    rng = np.random.default_rng(seed)
    R = restate.rodrigues(rng.normal(size=3) * 0.08)
    t = np.array([0.3, 0.05, 0.1]) + rng.normal(size=3) * 0.05
    X = np.stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(3, 10, n)], 1)
    x1 = X @ K.T
    p1 = x1[:, :2] / x1[:, 2:]
    X2 = X @ R.T + t
    x2 = X2 @ K.T
    p2 = x2[:, :2] / x2[:, 2:]
    p1 = p1 + rng.normal(size=p1.shape) * noise
    p2 = p2 + rng.normal(size=p2.shape) * noise
    out = np.zeros(n, bool)
    m = int(round(outlier_frac * n))
    if m:
        idx = rng.choice(n, m, replace=False)
        out[idx] = True
        p2[idx] = np.stack([rng.uniform(0, 640, m), rng.uniform(0, 480, m)], 1)
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    Ki = np.linalg.inv(K)
    F = Ki.T @ tx @ R @ Ki
    F = F / F[2, 2]
    p1, p2 = p1.astype(np.float32), p2.astype(np.float32)
    if m:  # labelled outliers sit well outside the 3 px epipolar gate (>= 20 px)
        for _ in range(100):
            bad = out & (fm_error(F.reshape(9), p1, p2) <= 400.0)
            if not bad.any():
                break
            k = int(bad.sum())
            p2[bad] = np.stack([rng.uniform(0, 640, k), rng.uniform(0, 480, k)], 1).astype(np.float32)
        out &= fm_error(F.reshape(9), p1, p2) > 400.0
    return p1, p2, F, out


def fm_error(F, p1, p2):
    """FMEstimatorCallback::computeError (float result)."""
    F = np.asarray(F, np.float64).reshape(9)
    x1, y1 = p1[:, 0].astype(np.float64), p1[:, 1].astype(np.float64)
    x2, y2 = p2[:, 0].astype(np.float64), p2[:, 1].astype(np.float64)
    a, b, c = F[0] * x1 + F[1] * y1 + F[2], F[3] * x1 + F[4] * y1 + F[5], F[6] * x1 + F[7] * y1 + F[8]
    s2, d2 = 1.0 / (a * a + b * b), x2 * a + y2 * b + c
    a, b, c = F[0] * x2 + F[3] * y2 + F[6], F[1] * x2 + F[4] * y2 + F[7], F[2] * x2 + F[5] * y2 + F[8]
    s1, d1 = 1.0 / (a * a + b * b), x1 * a + y1 * b + c
    return np.maximum(d1 * d1 * s1, d2 * d2 * s2).astype(np.float32)


def collinear(pts):
    i = len(pts) - 1
    eps = np.finfo(np.float32).eps
    for j in range(i):
        dx1, dy1 = float(pts[j][0]) - float(pts[i][0]), float(pts[j][1]) - float(pts[i][1])
        for k in range(j):
            dx2, dy2 = float(pts[k][0]) - float(pts[i][0]), float(pts[k][1]) - float(pts[i][1])
            if abs(dx2 * dy1 - dy2 * dx1) <= eps * (abs(dx1) + abs(dy1) + abs(dx2) + abs(dy2)):
                return True
    return False


def subsets(p1, p2, max_attempts):
    g, n = cv_rng(), len(p1)
    while True:
        for _ in range(max_attempts):
            idx = []
            while len(idx) < 7:
                v = next(g) % n
                if v not in idx:
                    idx.append(v)
            if not collinear(p1[idx]) and not collinear(p2[idx]):
                yield idx
                break
        else:
            yield None


def seven_point_numpy(a, b):
    """Independent 7-point: Hartley normalisation, numpy SVD null space, np.roots on det."""
    a, b = a.astype(np.float64), b.astype(np.float64)
    ca, cb = a.mean(0), b.mean(0)
    sa = math.sqrt(2) / np.mean(np.hypot(*(a - ca).T))
    sb = math.sqrt(2) / np.mean(np.hypot(*(b - cb).T))
    A0, B0 = (a - ca) * sa, (b - cb) * sb
    M = np.stack([B0[:, 0] * A0[:, 0], B0[:, 0] * A0[:, 1], B0[:, 0], B0[:, 1] * A0[:, 0], B0[:, 1] * A0[:, 1],
                  B0[:, 1], A0[:, 0], A0[:, 1], np.ones(7)], 1)
    V = np.linalg.svd(M)[2]
    f1, f2 = V[7].reshape(3, 3), V[8].reshape(3, 3)
    # det(l f1 + (1-l) f2) is a cubic in l: fit through 4 samples
    ls = np.array([-1.0, 0.0, 1.0, 2.0])
    coef = np.polyfit(ls, [np.linalg.det(l * f1 + (1 - l) * f2) for l in ls], 3)
    T1 = np.array([[sa, 0, -sa * ca[0]], [0, sa, -sa * ca[1]], [0, 0, 1]])
    T2 = np.array([[sb, 0, -sb * cb[0]], [0, sb, -sb * cb[1]], [0, 0, 1]])
    out = []
    for r in np.roots(coef):
        if abs(r.imag) > 1e-9 * max(1, abs(r.real)):
            continue
        F = T2.T @ (r.real * f1 + (1 - r.real) * f2) @ T1
        out.append(F / F[2, 2])
    return out


def replay(p1, p2, thr=3.0, conf=0.999, max_iters=1000):
    n = len(p1)
    if n >= 15:
        gen = subsets(p1, p2, 10000)
        niters, best, best_iter, bestF, it = max_iters, 0, -1, None, 0
        while it < niters:
            idx = next(gen)
            if idx is None:
                break
            for F in seven_point_numpy(p1[idx], p2[idx]):
                cnt = int((fm_error(F, p1, p2) <= np.float32(thr * thr)).sum())
                if cnt > max(best, 6):
                    best, best_iter, bestF = cnt, it, F
                    niters = ransac_update_num_iters(conf, (n - cnt) / n, 7, niters)
            it += 1
        return 2, it, best_iter, bestF
    gen = subsets(p1, p2, 1000)
    niters = max(ransac_update_num_iters(conf, 0.45, 7, max_iters), 3)
    best_med, best_iter, bestF = np.inf, -1, None
    for it in range(niters):
        idx = next(gen)
        for F in seven_point_numpy(p1[idx], p2[idx]):
            med = float(np.sort(fm_error(F, p1, p2))[n // 2])
            if med < best_med:
                best_med, best_iter, bestF = med, it, F
    return 3, niters, best_iter, bestF


@pytest.mark.parametrize("n,seed,out", [(60, 0, 0.0), (150, 1, 0.3), (400, 2, 0.5)])
def test_fundamental_known_answer(oracle, n, seed, out):
    p1, p2, F, outl = two_view(n, seed, outlier_frac=out)
    ok, Fo, mask, diag = oracle.find_fundamental(p1, p2)
    assert ok and diag[0] == 2
    # the RANSAC path returns the winning 7-point model (no refit), so its accuracy is that of a
    # minimal sample of float-rounded pixels: check consistency rather than 1e-6 agreement
    assert np.max(np.abs(Fo / np.linalg.norm(Fo) - F / np.linalg.norm(F))) < 1e-2
    # every true inlier kept; a winning 7-point subset may contain one outlier that its own model
    # fits exactly, so allow <= 1% labelled outliers inside the gate
    assert mask[~outl].all() and mask[outl].sum() <= max(1, n // 100)
    assert oracle.epipolar_error(p1[mask], p2[mask], Fo) < (1e-2 if not mask[outl].any() else 1.0)


@pytest.mark.parametrize("n,seed,noise,out", [(40, 3, 0.5, 0.2), (200, 4, 1.0, 0.4), (15, 5, 0.3, 0.0),
                                              (120, 6, 0.5, 0.6)])
def test_ransac_matches_numpy_replay(oracle, n, seed, noise, out):
    p1, p2, F, outl = two_view(n, seed, noise, out)
    ok, Fo, mask, diag = oracle.find_fundamental(p1, p2)
    method, iters, best_iter, Fr = replay(p1, p2)
    assert ok and diag[0] == method and diag[1] == iters and diag[2] == best_iter
    assert np.max(np.abs(Fo - Fr)) <= 1e-6 * np.abs(Fr).max()
    assert np.array_equal(mask, fm_error(Fo, p1, p2) <= np.float32(9.0))


@pytest.mark.parametrize("n,seed", [(14, 9), (14, 13)])
def test_lmeds_small_sets_match_numpy_replay(oracle, n, seed):
    # For n <= 13 the median (element n/2) is one of the 7 subset points, whose error is rounding
    # noise (~1e-20), so the winner is not a stable quantity; n = 14 is the first well-posed size.
    p1, p2, F, _ = two_view(n, seed, noise=0.5)
    ok, Fo, mask, diag = oracle.find_fundamental(p1, p2)
    method, iters, best_iter, Fr = replay(p1, p2)
    assert diag[0] == 3 and diag[1] == iters and diag[2] == best_iter
    assert np.max(np.abs(Fo - Fr)) <= 1e-6 * np.abs(Fr).max()
    med = float(np.sort(fm_error(Fr, p1, p2))[n // 2])
    sigma = max(2.5 * 1.4826 * (1 + 5.0 / (n - 7)) * math.sqrt(med), 0.001)
    m = fm_error(Fo, p1, p2) <= np.float32(sigma * sigma)
    assert ok == (m.sum() >= 7)
    if ok:
        assert np.array_equal(mask, m)


@pytest.mark.parametrize("n,seed", [(8, 7), (11, 8)])
def test_lmeds_tiny_sets_structure(oracle, n, seed):
    p1, p2, F, _ = two_view(n, seed, noise=0.5)
    ok, Fo, mask, diag = oracle.find_fundamental(p1, p2)
    assert diag[0] == 3 and diag[1] == max(ransac_update_num_iters(0.999, 0.45, 7, 1000), 3)
    assert ok == (diag[3] >= 7) and (not ok or mask.sum() == diag[3])


def test_fundamental_edges(oracle):
    p1, p2, F, _ = two_view(7, 10)
    ok, Fo, mask, diag = oracle.find_fundamental(p1, p2)   # n == 7: one 7-point solve
    assert diag[0] == 1 and ok and mask.all()
    assert np.max(np.abs(fm_error(Fo, p1, p2))) < 1e-3
    ok, _, _, diag = oracle.find_fundamental(p1[:6], p2[:6])  # n < 7: empty F
    assert not ok and diag[0] == 0
    # all points on one line in image 1: every subset is degenerate -> no model
    q1 = np.stack([np.linspace(0, 600, 30), np.linspace(0, 400, 30)], 1).astype(np.float32)
    ok, _, _, diag = oracle.find_fundamental(q1, p2[:1].repeat(30, 0) + np.arange(30)[:, None].astype(np.float32))
    assert not ok


def test_epipolar_error_formula(oracle):
    p1, p2, F, _ = two_view(50, 11, noise=1.0)
    x1 = np.c_[p1.astype(np.float64), np.ones(50)]
    x2 = np.c_[p2.astype(np.float64), np.ones(50)]
    Fx1 = x1 @ F.T
    d = np.abs(np.sum(x2 * Fx1, 1)) / np.hypot(Fx1[:, 0], Fx1[:, 1])
    assert abs(oracle.epipolar_error(p1, p2, F) - d.mean()) < 1e-12 * d.mean()
    assert oracle.epipolar_error(p1[:0], p2[:0], F) == 0


def test_fmat_verify_filters_matches_in_order(oracle):
    p1, p2, F, outl = two_view(120, 12, noise=0.3, outlier_frac=0.25)
    n = len(p1)
    kr = np.zeros(n + 5, oracle.KEYPOINT_DTYPE)
    kc = np.zeros(n + 3, oracle.KEYPOINT_DTYPE)
    perm_r, perm_c = np.random.default_rng(0).permutation(n + 5)[:n], np.random.default_rng(1).permutation(n + 3)[:n]
    kr["x"][perm_r], kr["y"][perm_r] = p1[:, 0], p1[:, 1]
    kc["x"][perm_c], kc["y"][perm_c] = p2[:, 0], p2[:, 1]
    good = np.zeros(n, oracle.MATCH_DTYPE)
    good["query_idx"], good["train_idx"] = perm_r, perm_c
    Fv, keep, err, diag = oracle.fmat_verify(kr, kc, good)
    ok, Fo, mask, _ = oracle.find_fundamental(p1, p2)
    assert Fv is not None and np.array_equal(Fv, Fo)
    assert np.array_equal(keep, np.flatnonzero(mask))
    assert err[0] == oracle.epipolar_error(p1, p2, Fo) and err[1] == oracle.epipolar_error(p1[mask], p2[mask], Fo)
    assert err[1] < err[0]
    Fv, keep, err, diag = oracle.fmat_verify(kr, kc, good[:5])  # too few: no F, nothing filtered
    assert Fv is None and np.array_equal(keep, np.arange(5)) and (err == 0).all()
