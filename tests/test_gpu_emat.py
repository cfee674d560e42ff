"""GPU parity for Slam::estimate_motion + the depth scale (A12, reference src/Slam.cpp:1193-1213,
73-207) through the C ABI.  The 5-point solver, Sampson scoring, recoverPose and the scale
estimators use only correctly rounded operations (+ - * / sqrt), shared with the CPU restatement,
so the outcome is compared exactly: RANSAC iterations, winning iteration, inlier and cheirality
counts, R, t and the scale."""
import numpy as np
import pytest

from test_oracle_emat import _depth_maps, two_view

pytestmark = pytest.mark.gpu


def _oracle_motion(oracle, p1, p2, d1, d2):
    ok_e, E, mask, fdiag = oracle.find_essential(p1, p2)
    ok, R, t, m, inl, good = oracle.estimate_motion(p1, p2)
    sc = oracle.estimate_scale(p1, p2, R, t, d1, d2) if ok and d1 is not None else -1.0
    return ok, R, t, sc, fdiag, inl, good


@pytest.mark.parametrize("n,seed,noise,out,depth", [(80, 0, 0.3, 0.2, 2), (200, 1, 0.5, 0.4, 2), (40, 2, 0.2, 0.0, 1),
                                                    (150, 3, 0.0, 0.3, 0), (400, 4, 0.7, 0.1, 2), (12, 5, 0.2, 0.5, 2)])
def test_estimate_motion_matches_oracle(vsctx, oracle, n, seed, noise, out, depth):
    p1, p2, R, t, X, outl = two_view(n, seed, noise=noise, outlier_frac=out)
    d1, d2 = _depth_maps(X, R, t, p1, p2)
    D1 = d1 if depth >= 1 else None
    D2 = d2 if depth >= 2 else None
    okg, Rg, tg, scg, dg = vsctx.estimate_motion(p1, p2, D1, D2)
    oko, Ro, to, sco, fdiag, inl, good = _oracle_motion(oracle, p1, p2, D1, D2)
    assert okg == oko
    assert dg[1] == fdiag[0] and dg[2] == fdiag[1] and dg[5] == n
    if fdiag[2] > 0:
        assert dg[3] == inl
    if oko:
        assert dg[4] == good
        assert np.array_equal(Rg, Ro) and np.array_equal(tg, to)
        assert scg == sco


def test_estimate_motion_edges(vsctx, oracle):
    p1, p2, R, t, X, outl = two_view(30, 6)
    assert not vsctx.estimate_motion(p1[:4], p2[:4])[0]
    ok, Rg, tg, sc, dg = vsctx.estimate_motion(p1, p2)  # no depth -> scale -1
    assert ok and sc == -1.0
    rng = np.random.default_rng(0)
    q = np.stack([rng.uniform(0, 640, 30), rng.uniform(0, 480, 30)], 1).astype(np.float32)
    assert vsctx.estimate_motion(q, q[::-1].copy())[0] == oracle.estimate_motion(q, q[::-1].copy())[0]
    with pytest.raises(RuntimeError):
        vsctx.estimate_motion(np.zeros((1024, 2), np.float32), np.zeros((1024, 2), np.float32))


def test_five_point_wave_equals_host(oracle):
    """The device's wave-parallel 5-point solver (emat.hip five_point_wave: coefficient columns, Gauss-Jordan
    columns and root intervals spread over the lanes) returns the host's models (emat_solvers.h five_point)
    bit for bit and in the same order: random, near-degenerate (q2 ~ q1) and real two-view subsets."""
    import ctypes

    import vslam_abi
    lib = vslam_abi.load_library()
    lib.vs_debug_five_point.restype = ctypes.c_int
    lib.vs_debug_five_point.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] + [ctypes.c_void_p] * 2
    rng = np.random.default_rng(11)
    count = 3000
    q1 = rng.uniform(-0.6, 0.6, (count, 10))
    q2 = rng.uniform(-0.6, 0.6, (count, 10))
    near = np.arange(count) % 7 == 0
    q2[near] = q1[near] + 1e-3 * rng.uniform(-1, 1, (int(near.sum()), 10))
    K = np.array([525.0, 525.0, 319.5, 239.5])
    for p in range(0, count, 5):  # every fifth: five correspondences of a noisy two-view scene
        a, b, _, _, _, _ = two_view(40, 100 + p, noise=0.3, outlier_frac=0.1)
        idx = rng.choice(40, 5, replace=False)
        q1[p] = ((a[idx] - K[2:]) / K[:2]).ravel()
        q2[p] = ((b[idx] - K[2:]) / K[:2]).ravel()
    E = np.zeros((count, 10, 9))
    nm = np.zeros(count, np.int32)
    assert lib.vs_debug_five_point(q1.ctypes.data, q2.ctypes.data, count, E.ctypes.data, nm.ctypes.data) == 0
    bad = []
    for p in range(count):
        Eh = oracle.five_point(q1[p], q2[p]).reshape(-1, 9)
        if nm[p] != len(Eh) or E[p, :nm[p]].view(np.uint64).tolist() != Eh.view(np.uint64).tolist():
            bad.append(p)
    assert nm.sum() > count, nm.sum()
    assert not bad, (len(bad), bad[:5])


@pytest.mark.parametrize("n,seed", [(5, 20), (6, 21), (7, 22), (64, 23), (65, 24)])
def test_estimate_motion_small_and_split_edges(vsctx, oracle, n, seed):
    """n == 5 (findEssentialMat's single kernel run on workgroup 0), n = 6, 7 (few points: the table's first rows),
    and 64 / 65 points around the split's 64 iterations: same outcome as the oracle."""
    p1, p2, R, t, X, outl = two_view(n, seed, noise=0.4, outlier_frac=0.3 if n > 10 else 0.0)
    okg, Rg, tg, scg, dg = vsctx.estimate_motion(p1, p2)
    oko, Ro, to, sco, fdiag, inl, good = _oracle_motion(oracle, p1, p2, None, None)
    assert okg == oko
    assert dg[1] == fdiag[0] and dg[2] == fdiag[1]
    if oko:
        assert np.array_equal(Rg, Ro) and np.array_equal(tg, to)


@pytest.mark.parametrize("split", [1, 2, 8])
def test_estimate_motion_small_split_continuation(vsctx, oracle, split):
    """The workgroup split forced small (1, 2, 8 workgroups = the first 8 / 16 / 64 iterations in parallel), so
    problems whose budget runs past the split finish in the last workgroup's continuation rounds (n = 400 at 50 %
    outliers runs 392 iterations): the same outcome as the oracle, iterations and winning iteration included."""
    import ctypes

    import vslam_abi
    lib = vslam_abi.load_library()
    lib.vs_debug_emat_split.restype = ctypes.c_int
    lib.vs_debug_emat_split.argtypes = [ctypes.c_int]
    assert lib.vs_debug_emat_split(split) == 0
    try:
        for n, seed, noise, out in [(400, 4, 0.7, 0.5), (200, 1, 0.5, 0.4), (80, 0, 0.3, 0.2), (6, 21, 0.4, 0.0)]:
            p1, p2, R, t, X, outl = two_view(n, seed, noise=noise, outlier_frac=out)
            d1, d2 = _depth_maps(X, R, t, p1, p2)
            okg, Rg, tg, scg, dg = vsctx.estimate_motion(p1, p2, d1, d2)
            oko, Ro, to, sco, fdiag, inl, good = _oracle_motion(oracle, p1, p2, d1, d2)
            assert okg == oko, (split, n)
            assert dg[1] == fdiag[0] and dg[2] == fdiag[1], (split, n, dg[:3], fdiag)
            if oko:
                assert np.array_equal(Rg, Ro) and np.array_equal(tg, to) and scg == sco, (split, n)
    finally:
        lib.vs_debug_emat_split(0)
