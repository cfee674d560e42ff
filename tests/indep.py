"""Independent numpy restatements of the geometric solvers on the hot path — TEST INFRASTRUCTURE.

They share no source with libvslam_hip.so or with oracle/ (which compiles the product's
csrc/*_solvers.h to check the device drivers bit for bit): every function here is written from the
published algorithm with numpy's own linear algebra (SVD / eigh / eig / lstsq / cholesky) and
Python's libm, so agreement with the product is tolerance-level, not bit-level.  They produce the
golden values of tests/golden/{pnp,fmat,emat,ba}.npz (tests/golden/make_golden.py) that both the
oracle (CPU suite) and the HIP path (GPU suite) are checked against.

  solve_pnp        Slam::solve_pnp (reference src/Slam.cpp:505-529): cv::solvePnPRansac — EPnP
                   (Lepetit, Moreno-Noguer, Fua 2009) hypotheses on cv::RNG 5-point subsets, the
                   RANSAC registrator's acceptance / iteration-update rules, Levenberg-Marquardt
                   refinement on the inliers; world pose R_cam^T, -R_cam^T t.
  find_fundamental cv::findFundamentalMat(FM_RANSAC, 3.0, 0.999) (Slam.cpp:880-910): 7-point
                   (null space + cubic), RANSAC for n >= 15, LMedS for 8 <= n <= 14.
  estimate_motion  Slam::estimate_motion (Slam.cpp:1193-1213): cv::findEssentialMat (5-point as a
                   cubic polynomial eigenvalue problem) + cv::recoverPose.
  local_ba         Optimizer::local_bundle_adjustment (Optimizer.cpp:296-575), dense numpy.
"""
import math

import numpy as np

K_TUM = (525.0, 525.0, 319.5, 239.5)
DBL_EPS = 2.220446049250313e-16
FLT_EPS = 1.1920928955078125e-07


# ------------------------------------------------------------------------------- cv::RNG
class CvRng:
    """cv::RNG: multiply-with-carry, state (uint64)-1 by default."""

    def __init__(self, state=(1 << 64) - 1):
        self.s = state

    def next(self):
        self.s = ((self.s & 0xFFFFFFFF) * 4164903690 + (self.s >> 32)) & ((1 << 64) - 1)
        return self.s & 0xFFFFFFFF

    def uniform(self, a, b):
        return a if a == b else self.next() % (b - a) + a


def ransac_update_num_iters(p, ep, model_points, max_iters):
    """cv::RANSACUpdateNumIters."""
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, 2.2250738585072014e-308)
    denom = 1.0 - (1.0 - ep) ** model_points
    if denom < 2.2250738585072014e-308:
        return 0
    num, denom = math.log(num), math.log(denom)
    if denom >= 0 or -num >= max_iters * (-denom):
        return max_iters
    return int(np.rint(num / denom))


def distinct_subset(rng, n, m):
    idx = []
    while len(idx) < m:
        v = rng.uniform(0, n)
        if v not in idx:
            idx.append(v)
    return idx


# ----------------------------------------------------------------------------- Rodrigues
def rod_v2m(r):
    r = np.asarray(r, np.float64).reshape(3)
    th = math.sqrt(float(r @ r))
    if th < DBL_EPS:
        return np.eye(3)
    k = r / th
    c, s = math.cos(th), math.sin(th)
    kx = np.array([[0.0, -k[2], k[1]], [k[2], 0.0, -k[0]], [-k[1], k[0], 0.0]])
    return c * np.eye(3) + (1.0 - c) * np.outer(k, k) + s * kx


def rod_m2v(R):
    """cv::Rodrigues(3x3 -> 3x1): nearest rotation by SVD, then the axis / angle."""
    U, _, Vt = np.linalg.svd(np.asarray(R, np.float64))
    R = U @ Vt
    rx, ry, rz = R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]
    s = math.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = min(max((np.trace(R) - 1.0) * 0.5, -1.0), 1.0)
    th = math.acos(c)
    if s < 1e-5:
        if c > 0:
            return np.zeros(3)
        v = np.sqrt(np.maximum((np.diag(R) + 1.0) * 0.5, 0.0))
        v[1] *= -1.0 if R[0, 1] < 0 else 1.0
        v[2] *= -1.0 if R[0, 2] < 0 else 1.0
        if abs(v[0]) < abs(v[1]) and abs(v[0]) < abs(v[2]) and (R[1, 2] > 0) != (v[1] * v[2] > 0):
            v[2] = -v[2]
        return v * (th / np.linalg.norm(v))
    return np.array([rx, ry, rz]) * (th / (2.0 * s))


# ------------------------------------------------------------------------------- PnP (A10)
def project(R, t, X, K):
    pc = X @ R.T + t
    return np.stack([K[0] * (pc[:, 0] / pc[:, 2]) + K[2], K[1] * (pc[:, 1] / pc[:, 2]) + K[3]], 1)


def reproj_err2(R, t, obj, img, K):
    """PnPRansacCallback::computeError: projectPoints (double -> float), float squared error."""
    proj = project(R, t, obj.astype(np.float64), K).astype(np.float32)
    d = img.astype(np.float32) - proj
    return d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]


def epnp(X, uv, K):
    """EPnP: control points from the PCA of X, barycentric alphas, the 4-dim null space of M^T M,
    the N = 4 / 2 / 3 beta approximations refined by 5 Gauss-Newton steps; the pose with the
    lowest mean reprojection error wins.  Returns (R, t) world -> camera or None."""
    X = np.asarray(X, np.float64)
    uv = np.asarray(uv, np.float64)
    n = len(X)
    c0 = X.mean(0)
    evals, evecs = np.linalg.eigh((X - c0).T @ (X - c0))
    # principal axes with their largest-magnitude component positive (the library's convention;
    # the signs are arbitrary in cv::SVD, but they decide the control points and so M)
    for c in range(3):
        if evecs[np.argmax(np.abs(evecs[:, c])), c] < 0:
            evecs[:, c] = -evecs[:, c]
    order = np.argsort(evals)[::-1]
    cw = [c0] + [c0 + math.sqrt(max(evals[o], 0.0) / n) * evecs[:, o] for o in order]
    cw = np.array(cw)
    CC = (cw[1:] - cw[0]).T
    if abs(np.linalg.det(CC)) < 1e-300:
        return None
    a123 = np.linalg.solve(CC, (X - c0).T).T
    alphas = np.concatenate([1.0 - a123.sum(1, keepdims=True), a123], 1)
    M = np.zeros((2 * n, 12))
    for i in range(n):
        for j in range(4):
            M[2 * i, 3 * j:3 * j + 3] = [alphas[i, j] * K[0], 0.0, alphas[i, j] * (K[2] - uv[i, 0])]
            M[2 * i + 1, 3 * j:3 * j + 3] = [0.0, alphas[i, j] * K[1], alphas[i, j] * (K[3] - uv[i, 1])]
    w, V = np.linalg.eigh(M.T @ M)
    v = [V[:, np.argsort(w)[k]] for k in range(4)]  # k-th smallest eigenvalue
    if n <= 5:
        # A 4- or 5-point M has a null space of dimension 12 - 2n >= 2, in which any solver's basis
        # is arbitrary (cv::SVD's follows rounding) and the N = 2 / 3 approximations depend on it.
        # The library takes the Householder QR basis of M^T (LAPACK's dgeqrf sign convention):
        # null vectors Q e_{2n}, Q e_{2n+1}, ..., then the eigenvectors of the smallest nonzero
        # eigenvalues; numpy's QR of the same M^T gives the same basis to rounding.
        Q, _ = np.linalg.qr(M.T, mode="complete")
        nz = 12 - 2 * n
        v = [Q[:, 2 * n + k] for k in range(nz)] + [V[:, np.argsort(w)[k]] for k in range(nz, 4)]
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    L = np.zeros((6, 10))
    rho = np.zeros(6)
    for j, (a, b) in enumerate(pairs):
        dv = [vk[3 * a:3 * a + 3] - vk[3 * b:3 * b + 3] for vk in v]
        d = lambda p, q: float(dv[p] @ dv[q])
        L[j] = [d(0, 0), 2 * d(0, 1), d(1, 1), 2 * d(0, 2), 2 * d(1, 2), d(2, 2), 2 * d(0, 3), 2 * d(1, 3),
                2 * d(2, 3), d(3, 3)]
        rho[j] = float((cw[a] - cw[b]) @ (cw[a] - cw[b]))

    def lsq(cols):
        return np.linalg.lstsq(L[:, cols], rho, rcond=None)[0]

    def betas(s):
        be = np.zeros(4)
        if s == 0:  # N = 4: B11 B12 B13 B14
            x = lsq([0, 1, 3, 6])
            b0 = math.sqrt(abs(x[0]))
            sg = -1.0 if x[0] < 0 else 1.0
            be[:] = [b0] + [sg * x[k] / b0 if b0 else 0.0 for k in (1, 2, 3)]
        else:       # N = 2: B11 B12 B22 ; N = 3: B11 B12 B22 B13 B23
            x = lsq([0, 1, 2] if s == 1 else [0, 1, 2, 3, 4])
            if x[0] < 0:
                b0, b1 = math.sqrt(-x[0]), (math.sqrt(-x[2]) if x[2] < 0 else 0.0)
            else:
                b0, b1 = math.sqrt(x[0]), (math.sqrt(x[2]) if x[2] > 0 else 0.0)
            if x[1] < 0:
                b0 = -b0
            be[:2] = b0, b1
            if s == 2:
                be[2] = x[3] / b0 if b0 else 0.0
        for _ in range(5):  # Gauss-Newton on the six distance constraints
            A = np.zeros((6, 4))
            r = np.zeros(6)
            for j in range(6):
                l = L[j]
                A[j] = [2 * l[0] * be[0] + l[1] * be[1] + l[3] * be[2] + l[6] * be[3],
                        l[1] * be[0] + 2 * l[2] * be[1] + l[4] * be[2] + l[7] * be[3],
                        l[3] * be[0] + l[4] * be[1] + 2 * l[5] * be[2] + l[8] * be[3],
                        l[6] * be[0] + l[7] * be[1] + l[8] * be[2] + 2 * l[9] * be[3]]
                q = [be[0] * be[0], be[0] * be[1], be[1] * be[1], be[0] * be[2], be[1] * be[2], be[2] * be[2],
                     be[0] * be[3], be[1] * be[3], be[2] * be[3], be[3] * be[3]]
                r[j] = rho[j] - float(l @ q)
            be = be + np.linalg.lstsq(A, r, rcond=None)[0]
        return be

    best = None
    for s in range(3):
        be = betas(s)
        ccs = sum(be[k] * v[k].reshape(4, 3) for k in range(4))
        pcs = alphas @ ccs
        if pcs[0, 2] < 0:
            pcs = -pcs
        pc0, pw0 = pcs.mean(0), X.mean(0)
        U, _, Vt = np.linalg.svd((pcs - pc0).T @ (X - pw0))
        R = U @ np.diag([1.0, 1.0, np.sign(np.linalg.det(U @ Vt)) or 1.0]) @ Vt
        t = pc0 - R @ pw0
        err = float(np.mean(np.linalg.norm(uv - project(R, t, X, K), axis=1)))
        if best is None or err < best[0]:
            best = (err, R, t)
    return best[1], best[2]


def pnp_lm(obj, img, p, K, max_iters=20, h=1e-6):
    """Levenberg-Marquardt over p = (rvec, tvec) on the inliers: rotation Jacobian by central
    differences, translation analytic, (J^T J with its diagonal scaled by 1 + lambda) d = -J^T r,
    lambda 1e-3, /10 on success (>= 1e-15), x10 on failure; stops on a relative step below
    DBL_EPSILON (solve) / FLT_EPSILON (accepted step) or lambda > 1e16."""
    X = obj.astype(np.float64)
    uv = img.astype(np.float64)

    def terms(q):
        R = rod_v2m(q[:3])
        t = q[3:]
        pc = X @ R.T + t
        iz = 1.0 / pc[:, 2]
        r = np.stack([K[0] * pc[:, 0] * iz + K[2], K[1] * pc[:, 1] * iz + K[3]], 1) - uv
        J = np.zeros((len(X), 2, 6))
        for k in range(3):
            e = np.zeros(3)
            e[k] = h
            J[:, :, k] = (project(rod_v2m(q[:3] + e), t, X, K) - project(rod_v2m(q[:3] - e), t, X, K)) / (2 * h)
        J[:, 0, 3] = K[0] * iz
        J[:, 0, 5] = -K[0] * pc[:, 0] * iz * iz
        J[:, 1, 4] = K[1] * iz
        J[:, 1, 5] = -K[1] * pc[:, 1] * iz * iz
        J = J.reshape(-1, 6)
        r = r.reshape(-1)
        return J.T @ J, J.T @ r, float(r @ r)

    p = np.asarray(p, np.float64).copy()
    A, g, cost = terms(p)
    lam, it = 1e-3, 0
    while it < max_iters:
        it += 1
        Ad = A.copy()
        Ad[np.diag_indices(6)] *= 1.0 + lam
        try:
            d = -np.linalg.solve(np.linalg.cholesky(Ad).T, np.linalg.solve(np.linalg.cholesky(Ad), g))
        except np.linalg.LinAlgError:
            lam *= 10
            continue
        if np.linalg.norm(d) <= DBL_EPS * np.linalg.norm(p):
            break
        cand = p + d
        A2, g2, c2 = terms(cand)
        if c2 < cost:
            step = np.linalg.norm(cand - p)
            p, A, g, cost = cand, A2, g2, c2
            lam = max(lam / 10, 1e-15)
            if step <= FLT_EPS * np.linalg.norm(p):
                break
        else:
            lam *= 10
            if lam > 1e16:
                break
    return p


def pnp_ransac(obj, img, iters=100, thr=8.0, conf=0.99, K=K_TUM):
    """cv::solvePnPRansac(useExtrinsicGuess = false, SOLVEPNP_ITERATIVE): returns (ok, rvec, tvec,
    inlier count, mask, (iterations run, winning iteration))."""
    obj = np.asarray(obj, np.float32)
    img = np.asarray(img, np.float32)
    n = len(obj)
    if n < 4:
        return False, None, None, 0, np.zeros(n, bool), (0, -1)
    mp = 4 if n == 4 else 5
    if n == mp:
        res = epnp(obj, img, K)
        if res is None:
            return False, None, None, 0, np.zeros(n, bool), (0, -1)
        return True, rod_m2v(res[0]), res[1], n, np.ones(n, bool), (0, -1)
    rng = CvRng()
    thr2 = np.float32(thr * thr)
    niters, best, best_iter, model = max(iters, 1), 0, -1, None
    it = 0
    while it < niters:
        idx = distinct_subset(rng, n, mp)
        res = epnp(obj[idx], img[idx], K)
        if res is not None:
            rv, tv = rod_m2v(res[0]), res[1]
            cnt = int(np.sum(reproj_err2(rod_v2m(rv), tv, obj, img, K) <= thr2))
            if cnt > max(best, mp - 1):
                best, best_iter, model = cnt, it, (rv, tv)
                niters = ransac_update_num_iters(conf, (n - cnt) / n, mp, niters)
        it += 1
    if model is None:
        return False, None, None, 0, np.zeros(n, bool), (it, best_iter)
    mask = reproj_err2(rod_v2m(model[0]), model[1], obj, img, K) <= thr2
    p = pnp_lm(obj[mask], img[mask], np.concatenate(model), K)
    return True, p[:3], p[3:], best, mask, (it, best_iter)


def solve_pnp(obj, img, ransac_iters=100, min_inliers=10, K=K_TUM):
    """Slam::solve_pnp (Slam.cpp:505-529): (success, R_world, t_world, inlier_count)."""
    if len(obj) < min_inliers:
        return False, None, None, 0
    ok, rv, tv, inl, mask, _ = pnp_ransac(obj, img, ransac_iters, float(np.float32(8.0)), 0.99, K)
    if not ok or inl < min_inliers:
        return False, None, None, 0
    Rc = rod_v2m(rv)
    return True, Rc.T, -Rc.T @ tv, inl


# ------------------------------------------------------------------------ F-matrix (A8)
def _have_collinear(x, y):
    """haveCollinearPoints for the last point of the subset."""
    i = len(x) - 1
    for j in range(i):
        dx1, dy1 = float(x[j]) - float(x[i]), float(y[j]) - float(y[i])
        for k in range(j):
            dx2, dy2 = float(x[k]) - float(x[i]), float(y[k]) - float(y[i])
            if abs(dx2 * dy1 - dy2 * dx1) <= FLT_EPS * (abs(dx1) + abs(dy1) + abs(dx2) + abs(dy2)):
                return True
    return False


def _f_subset(rng, p1, p2, n, attempts):
    for _ in range(attempts):
        idx = distinct_subset(rng, n, 7)
        if not _have_collinear(p1[idx, 0], p1[idx, 1]) and not _have_collinear(p2[idx, 0], p2[idx, 1]):
            return idx
    return None


def solve_cubic(c):
    """Real roots of c0 x^3 + c1 x^2 + c2 x + c3 in cv::solveCubic's order (trigonometric method)."""
    a0, a1, a2, a3 = c
    if a0 == 0:
        if a1 == 0:
            return [] if a2 == 0 else [-a3 / a2]
        d = a2 * a2 - 4 * a1 * a3
        if d < 0:
            return []
        d = math.sqrt(d)
        q1, q2 = (-a2 + d) * 0.5, (a2 + d) * -0.5
        r = [q1 / a1, a3 / q1] if abs(q1) > abs(q2) else [q2 / a1, a3 / q2]
        return r if d > 0 else r[:1]
    a1, a2, a3 = a1 / a0, a2 / a0, a3 / a0
    Q = (a1 * a1 - 3 * a2) / 9
    R = (a1 * (2 * a1 * a1 - 9 * a2) + 27 * a3) / 54
    if Q ** 3 - R * R >= 0:
        th = math.acos(R / math.sqrt(Q ** 3)) / 3
        return [-2 * math.sqrt(Q) * math.cos(th + k * 2 * math.pi / 3) - a1 / 3 for k in range(3)]
    e = (math.sqrt(R * R - Q ** 3) + abs(R)) ** (1.0 / 3)
    e = -e if R > 0 else e
    return [(e + Q / e) - a1 / 3]


def seven_point(x1, x2):
    """run7Point: Hartley normalisation, the null space of the 7 x 9 system parameterised by its
    last two unknowns (f7, f8) = (1, 0) / (0, 1), det(lambda F1 + mu F2) = 0, de-normalised and
    scaled so F(3,3) = 1."""
    x1 = x1.astype(np.float64)
    x2 = x2.astype(np.float64)
    m1, m2 = x1.mean(0), x2.mean(0)
    s1 = np.mean(np.linalg.norm(x1 - m1, axis=1))
    s2 = np.mean(np.linalg.norm(x2 - m2, axis=1))
    if s1 < FLT_EPS or s2 < FLT_EPS:
        return []
    s1, s2 = math.sqrt(2.0) / s1, math.sqrt(2.0) / s2
    a, b = (x1 - m1) * s1, (x2 - m2) * s2
    A = np.stack([b[:, 0] * a[:, 0], b[:, 0] * a[:, 1], b[:, 0], b[:, 1] * a[:, 0], b[:, 1] * a[:, 1], b[:, 1],
                  a[:, 0], a[:, 1], np.ones(7)], 1)
    try:
        sol = np.linalg.solve(A[:, :7], -A[:, 7:])
    except np.linalg.LinAlgError:
        return []
    f1 = np.concatenate([sol[:, 0], [1.0, 0.0]])
    f2 = np.concatenate([sol[:, 1], [0.0, 1.0]])
    f1 = f1 - f2
    F1, F2 = f1.reshape(3, 3), f2.reshape(3, 3)
    # det(x F1 + F2) as a cubic in x, coefficients by interpolation at four points
    xs = np.array([-1.0, 0.0, 1.0, 2.0])
    dets = [np.linalg.det(x * F1 + F2) for x in xs]
    c = np.linalg.solve(np.vander(xs, 4), dets)
    T1 = np.array([[s1, 0, -s1 * m1[0]], [0, s1, -s1 * m1[1]], [0, 0, 1.0]])
    T2 = np.array([[s2, 0, -s2 * m2[0]], [0, s2, -s2 * m2[1]], [0, 0, 1.0]])
    out = []
    for r in solve_cubic(list(c)):
        lam, mu = r, 1.0
        s = f1[8] * r + f2[8]
        if abs(s) > DBL_EPS:
            mu = 1.0 / s
            lam *= mu
        Fn = lam * F1 + mu * F2
        if abs(s) > DBL_EPS:
            Fn[2, 2] = 1.0
        F = T2.T @ Fn @ T1
        if abs(F[2, 2]) > FLT_EPS:
            F = F / F[2, 2]
        out.append(F)
    return out


def fm_error(F, p1, p2):
    """FMEstimatorCallback::computeError: max of the two squared point-line distances, float."""
    P1 = np.concatenate([p1.astype(np.float64), np.ones((len(p1), 1))], 1)
    P2 = np.concatenate([p2.astype(np.float64), np.ones((len(p2), 1))], 1)
    l2 = P1 @ F.T  # F x1
    l1 = P2 @ F    # F^T x2
    d2 = np.sum(P2 * l2, 1)
    e2 = d2 * d2 / (l2[:, 0] ** 2 + l2[:, 1] ** 2)
    e1 = d2 * d2 / (l1[:, 0] ** 2 + l1[:, 1] ** 2)
    return np.maximum(e1, e2).astype(np.float32)


def find_fundamental(p1, p2, thr=3.0, conf=0.999, max_iters=1000):
    """cv::findFundamentalMat(FM_RANSAC): (ok, F, mask, (method, iterations, winning iteration,
    inliers)); method 1 = n == 7, 2 = RANSAC, 3 = LMedS."""
    p1 = np.asarray(p1, np.float32).reshape(-1, 2)
    p2 = np.asarray(p2, np.float32).reshape(-1, 2)
    n = len(p1)
    none = (False, None, np.zeros(n, bool))
    if n == 7:
        Fs = seven_point(p1, p2)
        return (True, Fs[0], np.ones(n, bool), (1, 0, -1, n)) if Fs else none + ((1, 0, -1, 0),)
    if n < 8:
        return none + ((0, 0, -1, 0),)
    rng = CvRng()
    if n >= 15:
        thr2 = np.float32(thr * thr)
        niters, best, best_iter, bestF, it = max_iters, 0, -1, None, 0
        while it < niters:
            idx = _f_subset(rng, p1, p2, n, 10000)
            if idx is None:
                if it == 0:
                    return none + ((2, it, -1, 0),)
                break
            for F in seven_point(p1[idx], p2[idx]):
                cnt = int(np.sum(fm_error(F, p1, p2) <= thr2))
                if cnt > max(best, 6):
                    best, best_iter, bestF = cnt, it, F
                    niters = ransac_update_num_iters(conf, (n - cnt) / n, 7, niters)
            it += 1
        if bestF is None:
            return none + ((2, it, best_iter, 0),)
        mask = fm_error(bestF, p1, p2) <= thr2
        return True, bestF, mask, (2, it, best_iter, int(mask.sum()))
    niters = max(ransac_update_num_iters(conf, 0.45, 7, max_iters), 3)
    best_med, best_iter, bestF, it = np.inf, -1, None, 0
    while it < niters:
        idx = _f_subset(rng, p1, p2, n, 1000)
        if idx is None:
            if it == 0:
                return none + ((3, it, -1, 0),)
            break
        for F in seven_point(p1[idx], p2[idx]):
            med = float(np.sort(fm_error(F, p1, p2))[n // 2])
            if med < best_med:
                best_med, best_iter, bestF = med, it, F
        it += 1
    if bestF is None:
        return none + ((3, it, best_iter, 0),)
    sigma = max(2.5 * 1.4826 * (1 + 5.0 / (n - 7)) * math.sqrt(best_med), 0.001)
    mask = fm_error(bestF, p1, p2) <= np.float32(sigma * sigma)
    if mask.sum() < 7:
        return False, None, np.zeros(n, bool), (3, it, best_iter, int(mask.sum()))
    return True, bestF, mask, (3, it, best_iter, int(mask.sum()))


# ------------------------------------------------------------------------ E-matrix (A12)
def _mono_cubic():
    """Monomials of degree <= 3 in (x, y, z) as exponent triples."""
    return [(a, b, c) for a in range(4) for b in range(4) for c in range(4) if a + b + c <= 3]


def five_point(q1, q2):
    """Essential matrices from 5 normalised correspondences: E = x E0 + y E1 + z E2 + E3 over the
    null space (SVD), the ten cubic constraints det E = 0 and 2 E E^T E - tr(E E^T) E = 0 written
    as polynomials in (x, y) with coefficients in z, C(z) m(x, y) = 0 (m = the 10 monomials of
    degree <= 3 in x, y), solved as the cubic polynomial eigenvalue problem in z; x, y from the
    eigenvector.  Unit Frobenius norm."""
    A = np.stack([q2[:, 0] * q1[:, 0], q2[:, 0] * q1[:, 1], q2[:, 0], q2[:, 1] * q1[:, 0], q2[:, 1] * q1[:, 1],
                  q2[:, 1], q1[:, 0], q1[:, 1], np.ones(5)], 1)
    Eb = np.linalg.svd(A)[2][5:].reshape(4, 3, 3)  # basis E0..E3
    # polynomial matrices: entries are dicts {(a, b, c): coef} over x, y, z
    def lin(i, j):
        return {(1, 0, 0): Eb[0, i, j], (0, 1, 0): Eb[1, i, j], (0, 0, 1): Eb[2, i, j], (0, 0, 0): Eb[3, i, j]}

    def mul(p, q):
        out = {}
        for ea, ca in p.items():
            for eb, cb in q.items():
                e = (ea[0] + eb[0], ea[1] + eb[1], ea[2] + eb[2])
                out[e] = out.get(e, 0.0) + ca * cb
        return out

    def add(p, q, s=1.0):
        out = dict(p)
        for e, c in q.items():
            out[e] = out.get(e, 0.0) + s * c
        return out

    E = [[lin(i, j) for j in range(3)] for i in range(3)]
    det = {}
    for (i, j, k), s in (((0, 1, 2), 1), ((1, 2, 0), 1), ((2, 0, 1), 1), ((0, 2, 1), -1), ((1, 0, 2), -1),
                         ((2, 1, 0), -1)):
        det = add(det, mul(mul(E[0][i], E[1][j]), E[2][k]), s)
    EEt = [[{} for _ in range(3)] for _ in range(3)]
    for i in range(3):
        for j in range(3):
            for k in range(3):
                EEt[i][j] = add(EEt[i][j], mul(E[i][k], E[j][k]))
    tr = add(add(EEt[0][0], EEt[1][1]), EEt[2][2])
    eqs = [det]
    for i in range(3):
        for j in range(3):
            s = {}
            for k in range(3):
                s = add(s, mul(EEt[i][k], E[k][j]))
            eqs.append(add(mul(s, {(0, 0, 0): 2.0}), mul(tr, E[i][j]), -1.0))
    xy = [(a, b) for a in range(4) for b in range(4) if a + b <= 3]  # 10 monomials in x, y
    C = np.zeros((4, 10, 10))  # C[d] multiplies z^d
    for r, eq in enumerate(eqs):
        for (a, b, c), v in eq.items():
            C[c, r, xy.index((a, b))] += v
    # companion linearisation of C0 + z C1 + z^2 C2 + z^3 C3
    Z = np.zeros((10, 10))
    I = np.eye(10)
    Aa = np.block([[Z, I, Z], [Z, Z, I], [-C[0], -C[1], -C[2]]])
    Bb = np.block([[I, Z, Z], [Z, I, Z], [Z, Z, C[3]]])
    import scipy.linalg
    ab, V = scipy.linalg.eig(Aa, Bb, homogeneous_eigvals=True)
    sols = []
    ix, iy, i1 = xy.index((1, 0)), xy.index((0, 1)), xy.index((0, 0))
    for k in range(ab.shape[1]):
        if abs(ab[1, k]) < 1e-12 * abs(ab[0, k]):
            continue  # infinite eigenvalue (C3 is rank one)
        z = ab[0, k] / ab[1, k]
        if abs(z.imag) > 1e-8 * max(1.0, abs(z.real)):
            continue
        m = V[:10, k]
        if abs(m[i1]) < 1e-12:
            continue
        x, y = (m[ix] / m[i1]).real, (m[iy] / m[i1]).real
        Em = x * Eb[0] + y * Eb[1] + z.real * Eb[2] + Eb[3]
        sols.append((z.real, Em / np.linalg.norm(Em)))
    sols.sort(key=lambda s: s[0])
    return [E for _, E in sols]


def sampson(E, q1, q2):
    """EMEstimatorCallback::computeError: Sampson distance, float."""
    P1 = np.concatenate([q1, np.ones((len(q1), 1))], 1)
    P2 = np.concatenate([q2, np.ones((len(q2), 1))], 1)
    Ex1 = P1 @ E.T
    Etx2 = P2 @ E
    num = np.sum(P2 * Ex1, 1) ** 2
    return (num / (Ex1[:, 0] ** 2 + Ex1[:, 1] ** 2 + Etx2[:, 0] ** 2 + Etx2[:, 1] ** 2)).astype(np.float32)


def find_essential(p1, p2, K=K_TUM, prob=0.999, thr_px=1.0, max_iters=1000):
    """cv::findEssentialMat(RANSAC): (ok, E, mask, (iterations, winning iteration, inliers))."""
    p1 = np.asarray(p1, np.float32).reshape(-1, 2).astype(np.float64)
    p2 = np.asarray(p2, np.float32).reshape(-1, 2).astype(np.float64)
    n = len(p1)
    if n < 5:
        return False, None, np.zeros(n, bool), (0, -1, 0)
    q1 = (p1 - [K[2], K[3]]) / [K[0], K[1]]
    q2 = (p2 - [K[2], K[3]]) / [K[0], K[1]]
    thr = thr_px / ((K[0] + K[1]) / 2)
    thr2 = np.float32(thr * thr)
    if n == 5:
        Es = five_point(q1, q2)
        return (True, Es[0], np.ones(n, bool), (0, -1, n)) if Es else (False, None, np.zeros(n, bool), (0, -1, 0))
    rng = CvRng()
    niters, best, best_iter, bestE, it = max_iters, 0, -1, None, 0
    while it < niters:
        idx = distinct_subset(rng, n, 5)
        for E in five_point(q1[idx], q2[idx]):
            cnt = int(np.sum(sampson(E, q1, q2) <= thr2))
            if cnt > max(best, 4):
                best, best_iter, bestE = cnt, it, E
                niters = ransac_update_num_iters(prob, (n - cnt) / n, 5, niters)
        it += 1
    if bestE is None:
        return False, None, np.zeros(n, bool), (it, best_iter, 0)
    mask = sampson(bestE, q1, q2) <= thr2
    return True, bestE, mask, (it, best_iter, int(mask.sum()))


def recover_pose(E, p1, p2, mask, K=K_TUM, dist=50.0):
    """cv::recoverPose: decomposeEssentialMat, linear triangulation, cheirality with the distance
    threshold; the combination with the most good points wins (R1 t, R2 t, R1 -t, R2 -t order)."""
    p1 = np.asarray(p1, np.float32).reshape(-1, 2).astype(np.float64)
    p2 = np.asarray(p2, np.float32).reshape(-1, 2).astype(np.float64)
    q1 = (p1 - [K[2], K[3]]) / [K[0], K[1]]
    q2 = (p2 - [K[2], K[3]]) / [K[0], K[1]]
    U, _, Vt = np.linalg.svd(E)
    if np.linalg.det(U) < 0:
        U = -U
    if np.linalg.det(Vt) < 0:
        Vt = -Vt
    W = np.array([[0.0, 1, 0], [-1, 0, 0], [0, 0, 1]])
    R1, R2, t = U @ W @ Vt, U @ W.T @ Vt, U[:, 2]
    cands = [(R1, t), (R2, t), (R1, -t), (R2, -t)]
    goods, masks = [], []
    for R, tt in cands:
        P1 = np.hstack([R, tt[:, None]])
        m = np.zeros(len(q1), bool)
        for i in range(len(q1)):
            if mask is not None and not mask[i]:
                continue
            A = np.stack([q1[i, 0] * np.array([0, 0, 1.0, 0]) - [1.0, 0, 0, 0],
                          q1[i, 1] * np.array([0, 0, 1.0, 0]) - [0, 1.0, 0, 0],
                          q2[i, 0] * P1[2] - P1[0], q2[i, 1] * P1[2] - P1[1]])
            Q = np.linalg.svd(A)[2][-1]
            if not Q[2] * Q[3] > 0:
                continue
            X = Q[:3] / Q[3]
            z2 = R[2] @ X + tt[2]
            m[i] = X[2] < dist and 0 < z2 < dist
        goods.append(int(m.sum()))
        masks.append(m)
    k = int(np.argmax(goods))  # first maximum
    return goods[k], cands[k][0], cands[k][1], masks[k]


def estimate_motion(p1, p2, K=K_TUM):
    """Slam::estimate_motion (Slam.cpp:1193-1213): (ok, R, t, mask, inliers, good)."""
    n = len(p1)
    if n < 5:
        return False, None, None, None, 0, 0
    ok, E, mask, _ = find_essential(p1, p2, K)
    if not ok:
        return False, None, None, mask, 0, 0
    inl = int(mask.sum())
    if inl < 15:
        return False, None, None, mask, inl, 0
    good, R, t, m2 = recover_pose(E, p1, p2, mask, K)
    if good < 15 or abs(np.linalg.det(R) - 1.0) > 0.01:
        return False, R, t, m2, inl, good
    return True, R, t, m2, inl, good


# ------------------------------------------------------------------------ local BA (A14)
def local_ba(R_world, t_world, P, obs_kf, obs_pt, obs_uv, K=K_TUM, max_iter=15, huber=5.0):
    """Optimizer::local_bundle_adjustment's LM (Optimizer.cpp:250-575) on a gathered window, with a
    dense Schur complement: per observation the Huber-weighted (sqrt-scaled) residual, the
    analytic point / translation Jacobian and the forward-difference (eps 1e-6) rotation Jacobian;
    Hpp += 1e10 I; S and Hmm diagonals x (1 + lambda); Hmm^-1 (zero when |det| < 1e-20); dense
    solve; back-substitution; accept on a lower Huber cost (lambda = max(1e-7, lambda / 2), stop
    below a 1e-4 relative change), else lambda x 5 (stop above 1e6).  Returns (R, t, P, rms before,
    rms after, (iterations, accepted))."""
    fx, fy, cx, cy = K
    N, M = len(R_world), len(P)
    rv = [rod_m2v(R) for R in np.asarray(R_world, np.float64)]
    tv = [np.array(t, np.float64) for t in t_world]
    P = np.array(P, np.float64)
    obs = list(zip(np.asarray(obs_kf), np.asarray(obs_pt), np.asarray(obs_uv, np.float64)))
    if N < 2 or len(obs) < 20 or M < 10:
        return np.array(R_world), np.array(t_world), P, 0.0, 0.0, (0, 0)

    def proj(R, t, X):  # project_fn (:267-282); callers treat u < 0 like "behind" ((-1, -1))
        pc = R.T @ (X - t)
        if pc[2] < 1e-6:
            return None
        p = np.array([fx * pc[0] / pc[2] + cx, fy * pc[1] / pc[2] + cy])
        return None if p[0] < 0 else p

    def rms(rv_, tv_, P_):
        Rs = [rod_v2m(r) for r in rv_]
        s = 0.0
        for k, j, uv in obs:
            p = proj(Rs[k], tv_[k], P_[j])
            if p is not None:
                s += float(np.sum((p - uv) ** 2))
        return math.sqrt(s / len(obs))

    before = rms(rv, tv, P)
    lam, iters, accepted = 1e-4, 0, 0
    for _ in range(max_iter):
        iters += 1
        Rs = [rod_v2m(r) for r in rv]
        Hpp = np.zeros((N, 6, 6))
        bp = np.zeros((N, 6))
        Hmm = np.zeros((M, 3, 3))
        bm = np.zeros((M, 3))
        Hpm = {}
        cost = 0.0
        for k, j, uv in obs:
            d = P[j] - tv[k]
            pc = Rs[k].T @ d
            if pc[2] < 1e-6:
                continue
            iz = 1.0 / pc[2]
            up = np.array([fx * pc[0] * iz + cx, fy * pc[1] * iz + cy])
            r = up - uv
            rn = math.sqrt(float(r @ r))
            w = huber / rn if rn > huber else 1.0
            sw = math.sqrt(w)
            cost += w * float(r @ r)
            dproj = np.array([[fx * iz, 0.0, -fx * pc[0] * iz * iz], [0.0, fy * iz, -fy * pc[1] * iz * iz]])
            Jm = dproj @ Rs[k].T * sw
            Jr = np.zeros((2, 3))
            for a in range(3):
                e = np.zeros(3)
                e[a] = 1e-6
                pp = rod_v2m(rv[k] + e).T @ d
                if pp[2] < 1e-6:
                    continue
                Jr[:, a] = (np.array([fx * pp[0] / pp[2] + cx, fy * pp[1] / pp[2] + cy]) - up) / 1e-6 * sw
            Jp = np.hstack([Jr, -Jm])
            Hpp[k] += Jp.T @ Jp
            bp[k] += Jp.T @ (r * sw)
            Hmm[j] += Jm.T @ Jm
            bm[j] += Jm.T @ (r * sw)
            Hpm[(k, j)] = Hpm.get((k, j), 0.0) + Jp.T @ Jm
        S = np.zeros((6 * N, 6 * N))
        bs = np.zeros(6 * N)
        for k in range(N):
            S[6 * k:6 * k + 6, 6 * k:6 * k + 6] = Hpp[k] + 1e10 * np.eye(6)
            bs[6 * k:6 * k + 6] = bp[k]
        S[np.diag_indices(6 * N)] *= 1.0 + lam
        Hinv = np.zeros((M, 3, 3))
        observers = [[] for _ in range(M)]
        for (k, j) in Hpm:
            observers[j].append(k)
        for j in range(M):
            Hd = Hmm[j].copy()
            Hd[np.diag_indices(3)] *= 1.0 + lam
            if abs(np.linalg.det(Hd)) < 1e-20:
                continue
            Hinv[j] = np.linalg.inv(Hd)
            for ka in observers[j]:
                HaHi = Hpm[(ka, j)] @ Hinv[j]
                bs[6 * ka:6 * ka + 6] -= HaHi @ bm[j]
                for kb in observers[j]:
                    S[6 * ka:6 * ka + 6, 6 * kb:6 * kb + 6] -= HaHi @ Hpm[(kb, j)].T
        try:
            dp = np.linalg.solve(S, -bs)
        except np.linalg.LinAlgError:
            lam *= 10
            continue
        Pn = P.copy()
        for j in range(M):
            rhs = -bm[j].copy()
            for k in observers[j]:
                rhs -= Hpm[(k, j)].T @ dp[6 * k:6 * k + 6]
            Pn[j] = P[j] + Hinv[j] @ rhs
        rvn = [rv[k] + dp[6 * k:6 * k + 3] for k in range(N)]
        tvn = [tv[k] + dp[6 * k + 3:6 * k + 6] for k in range(N)]
        Rn = [rod_v2m(r) for r in rvn]
        new = 0.0
        for k, j, uv in obs:
            p = proj(Rn[k], tvn[k], Pn[j])
            if p is None:
                new += 100.0
                continue
            d2 = float(np.sum((p - uv) ** 2))
            rn = math.sqrt(d2)
            new += (huber / rn if rn > huber else 1.0) * d2
        if new < cost:
            rv, tv, P = rvn, tvn, Pn
            accepted += 1
            lam = max(1e-7, lam * 0.5)
            if (cost - new) / (cost + 1e-10) < 1e-4:
                break
        else:
            lam *= 5.0
            if lam > 1e6:
                break
    after = rms(rv, tv, P)
    Rout = np.array(R_world, np.float64).copy()
    tout = np.array(t_world, np.float64).copy()
    for k in range(1, N):  # Optimizer.cpp:584-588: keyframe 0 stays
        Rout[k] = rod_v2m(rv[k])
        tout[k] = tv[k]
    return Rout, tout, P, before, after, (iters, accepted)


# ------------------------------------------------------------- depth scale (A12, Slam.cpp:73-207)
def estimate_scale(p1, p2, R, t, depth1, depth2, K=K_TUM, dmin=np.float32(0.1), dmax=np.float32(10.0)):
    """Slam::estimate_scale_from_depth with the single-depth fallback (estimate_scale_single_depth):
    per match s = (P2 - R P1) . t from both depth maps, kept in (0.001, 50), IQR filter, median;
    -1 when no scale is found."""
    fx, fy, cx, cy = K
    p1 = np.asarray(p1, np.float32).reshape(-1, 2)
    p2 = np.asarray(p2, np.float32).reshape(-1, 2)
    h, w = depth1.shape

    def px(p):  # std::round on the float coordinate (half away from zero)
        return int(math.floor(float(p) + 0.5)) if p >= 0 else -int(math.floor(-float(p) + 0.5))

    def single():
        sc = []
        for a, b in zip(p1, p2):
            x1, y1 = px(a[0]), px(a[1])
            if not (0 <= x1 < w and 0 <= y1 < h):
                continue
            d1 = depth1[y1, x1]
            if d1 <= dmin or d1 > dmax:
                continue
            P1 = np.array([(float(a[0]) - cx) * float(d1) / fx, (float(a[1]) - cy) * float(d1) / fy, float(d1)])
            RP = R @ P1
            ax = (float(b[0]) - cx) / fx
            den = t[0] - ax * t[2]
            if abs(den) > 1e-4:
                s = (ax * RP[2] - RP[0]) / den
                if 0.001 < s < 100.0:
                    sc.append(s)
            by = (float(b[1]) - cy) / fy
            den = t[1] - by * t[2]
            if abs(den) > 1e-4:
                s = (by * RP[2] - RP[1]) / den
                if 0.001 < s < 100.0:
                    sc.append(s)
        return sorted(sc)[len(sc) // 2] if len(sc) >= 10 else -1.0

    if depth1 is None:
        return -1.0
    if depth2 is None:
        return single()
    sc = []
    for a, b in zip(p1, p2):
        x1, y1, x2, y2 = px(a[0]), px(a[1]), px(b[0]), px(b[1])
        if not (0 <= x1 < w and 0 <= y1 < h and 0 <= x2 < w and 0 <= y2 < h):
            continue
        d1, d2 = depth1[y1, x1], depth2[y2, x2]
        if d1 <= dmin or d1 > dmax or d2 <= dmin or d2 > dmax:
            continue
        P1 = np.array([(float(a[0]) - cx) * float(d1) / fx, (float(a[1]) - cy) * float(d1) / fy, float(d1)])
        P2 = np.array([(float(b[0]) - cx) * float(d2) / fx, (float(b[1]) - cy) * float(d2) / fy, float(d2)])
        s = float((P2 - R @ P1) @ t)
        if 0.001 < s < 50.0:
            sc.append(s)
    if len(sc) < 10:
        return single()
    sc.sort()
    q1, q3 = sc[len(sc) // 4], sc[3 * len(sc) // 4]
    lo, hi = q1 - 1.5 * (q3 - q1), q3 + 1.5 * (q3 - q1)
    f = [s for s in sc if lo <= s <= hi]
    return sorted(f)[len(f) // 2] if f else sc[len(sc) // 2]
