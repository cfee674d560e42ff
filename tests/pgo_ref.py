"""numpy restatement of Optimizer::pose_graph_optimize (reference src/Optimizer.cpp:654-863) under
g2o's conventions (EdgeSE3 error = (t, unit quaternion xyz with w >= 0) of Z^-1 Ta^-1 Tb, update
T <- T exp(dx) with dx = (t, quaternion xyz), OptimizationAlgorithmLevenberg's lambda schedule),
written independently of oracle/orc_pgo.cpp and csrc/pgo.hip (scipy's quaternion conversion,
numpy's Cholesky).  Test infrastructure only."""
import numpy as np
from scipy.spatial.transform import Rotation

STEP = 1e-6


def iso(R, t):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


def qvec(R):
    q = Rotation.from_matrix(R).as_quat()  # x y z w, unit
    return -q[:3] if q[3] < 0 else q[:3]


def exp_mqt(v):
    q = v[3:]
    w = 1.0 - q @ q
    if w < 0:
        R = np.eye(3)
    else:
        R = Rotation.from_quat([q[0], q[1], q[2], np.sqrt(w)]).as_matrix()
    return iso(R, v[:3])


def err(Zi, Ta, Tb):
    D = Zi @ np.linalg.inv(Ta) @ Tb
    return np.concatenate([D[:3, 3], qvec(D[:3, :3])])


def optimize(R, t, loops=(), gravity=None, height=0.0, iters=20):
    N = len(R)
    P = [iso(R[i], t[i]) for i in range(N)]
    edges = []
    om_odo = np.array([1 / 0.05 ** 2] * 3 + [1 / 0.02 ** 2] * 3)
    for i in range(N - 1):
        edges.append((i, i + 1, np.linalg.inv(np.linalg.inv(P[i]) @ P[i + 1]), om_odo))
    for a, b, Rr, tr, st, sr in loops:
        edges.append((a, b, np.linalg.inv(iso(Rr, tr)), np.array([1 / st ** 2] * 3 + [1 / sr ** 2] * 3)))
    hinfo = 1 / 0.005 ** 2
    g = None if gravity is None else np.asarray(gravity, float)

    def chi2(Q):
        c = sum(e @ (w * e) for e, w in ((err(Z, Q[a], Q[b]), w) for a, b, Z, w in edges))
        if g is not None:
            c += sum((g @ Q[v][:3, 3] - height) ** 2 * hinfo for v in range(1, N))
        return c

    n = 6 * (N - 1)
    chi = chi2(P)
    lam, ni = 0.0, 2.0
    for it in range(iters):
        H = np.zeros((n, n))
        bvec = np.zeros(n)
        for a, b, Z, w in edges:
            e0 = err(Z, P[a], P[b])
            J = np.zeros((6, 12))
            for c in range(12):
                dx = np.zeros(6)
                dx[c % 6] = STEP
                Tp = (P[a] if c < 6 else P[b]) @ exp_mqt(dx)
                dx[c % 6] = -STEP
                Tm = (P[a] if c < 6 else P[b]) @ exp_mqt(dx)
                ep = err(Z, Tp, P[b]) if c < 6 else err(Z, P[a], Tp)
                em = err(Z, Tm, P[b]) if c < 6 else err(Z, P[a], Tm)
                J[:, c] = (ep - em) / (2 * STEP)
            for s1, v1 in ((0, a), (1, b)):
                if v1 == 0:
                    continue
                J1 = J[:, 6 * s1:6 * s1 + 6]
                bvec[6 * (v1 - 1):6 * v1] -= J1.T @ (w * e0)
                for s2, v2 in ((0, a), (1, b)):
                    if v2 == 0:
                        continue
                    H[6 * (v1 - 1):6 * v1, 6 * (v2 - 1):6 * v2] += J1.T @ (w[:, None] * J[:, 6 * s2:6 * s2 + 6])
        if g is not None:
            for v in range(1, N):
                Jh = np.zeros(6)
                for c in range(6):
                    dx = np.zeros(6)
                    dx[c] = STEP
                    ep = g @ (P[v] @ exp_mqt(dx))[:3, 3] - height
                    dx[c] = -STEP
                    em = g @ (P[v] @ exp_mqt(dx))[:3, 3] - height
                    Jh[c] = (ep - em) / (2 * STEP)
                e = g @ P[v][:3, 3] - height
                sl = slice(6 * (v - 1), 6 * v)
                bvec[sl] -= Jh * hinfo * e
                H[sl, sl] += hinfo * np.outer(Jh, Jh)
        if it == 0:
            lam, ni = 1e-5 * np.max(np.abs(np.diag(H))), 2.0
        qmax, rho = 0, 0.0
        while True:
            x = np.linalg.solve(H + lam * np.eye(n), bvec)
            Pt = [P[0]] + [P[v] @ exp_mqt(x[6 * (v - 1):6 * v]) for v in range(1, N)]
            tchi = chi2(Pt)
            rho = (chi - tchi) / (x @ (lam * x + bvec) + 1e-3)
            if rho > 0 and np.isfinite(tchi):
                lam *= max(1 / 3, min(1 - (2 * rho - 1) ** 3, 2 / 3))
                ni = 2.0
                chi = tchi
                P = Pt
            else:
                lam *= ni
                ni *= 2
            qmax += 1
            if not (rho < 0 and qmax < 10):
                break
        if qmax == 10 or rho == 0 or not np.isfinite(lam):
            break
    return np.array([T[:3, :3] for T in P]), np.array([T[:3, 3] for T in P]), chi


def chain_problem(N, seed, loop_every=0):
    """A noisy open chain of N keyframe poses along a circle and (optionally) loop constraints tying
    vertex i to vertex N - 1 - ... with the ground-truth relative pose."""
    rng = np.random.default_rng(seed)
    gt = []
    for i in range(N):
        a = 2 * np.pi * i / N
        Rg = Rotation.from_euler("y", a).as_matrix()
        gt.append(iso(Rg, [np.cos(a) * 2, 0.4, np.sin(a) * 2]))
    est = [gt[0]]
    for i in range(1, N):
        rel = np.linalg.inv(gt[i - 1]) @ gt[i]
        noise = iso(Rotation.from_rotvec(rng.normal(0, 0.01, 3)).as_matrix(), rng.normal(0, 0.02, 3))
        est.append(est[-1] @ rel @ noise)
    loops = []
    if loop_every:
        for j in range(loop_every, N, loop_every):
            rel = np.linalg.inv(gt[0]) @ gt[j]
            loops.append((0 if j < N // 2 else j - loop_every // 2, j, None, None, 0.03, 0.01))
        loops = [(a, b, (np.linalg.inv(gt[a]) @ gt[b])[:3, :3], (np.linalg.inv(gt[a]) @ gt[b])[:3, 3], st, sr)
                 for a, b, _, _, st, sr in loops]
    R = np.array([T[:3, :3] for T in est])
    t = np.array([T[:3, 3] for T in est])
    return R, t, loops, gt
