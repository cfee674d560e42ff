"""GPU parity for Slam::solve_pnp (A10, reference src/Slam.cpp:505-529) through the C ABI.

The RANSAC outcome (success, inlier count, inlier mask, iterations run, winning iteration, LM
iteration counts) must equal the oracle's exactly; the refined world pose agrees to 1e-9 (the
LM normal equations are summed in a different order on the device)."""
import numpy as np
import pytest

from test_oracle_pnp import pnp_problem, rot_angle

pytestmark = pytest.mark.gpu

CASES = [(50, 0, 0.0, 0.0, 100, 10), (120, 1, 0.5, 0.3, 300, 15), (300, 2, 1.0, 0.5, 300, 15),
         (2000, 3, 0.7, 0.4, 100, 10), (40, 4, 0.5, 0.7, 100, 10), (12, 5, 0.3, 0.0, 100, 10)]


def _check_against_oracle(oracle, g, obj, img, iters, min_inl):
    ok_o, rv, tv, inl_o, mask_o, diag_o = oracle.pnp_ransac(obj, img, iters)
    succ_o, Rw_o, tw_o, cnt_o = oracle.solve_pnp(obj, img, iters, min_inl)
    succ, Rw, tw, cnt, mask, diag = g
    assert succ == succ_o and cnt == cnt_o
    if len(obj) >= min_inl:
        assert np.array_equal(diag[:2], diag_o[:2])
        if ok_o:
            assert np.array_equal(mask, mask_o)
    if succ:
        assert np.array_equal(diag, diag_o)
        assert np.max(np.abs(Rw - Rw_o)) < 1e-9 and np.max(np.abs(tw - tw_o)) < 1e-9


@pytest.mark.parametrize("n,seed,noise,out,iters,min_inl", CASES)
def test_solve_pnp_matches_oracle(vsctx, oracle, n, seed, noise, out, iters, min_inl):
    obj, img, R, t, outl = pnp_problem(n, seed, noise=noise, outlier_frac=out)
    g = vsctx.solve_pnp(obj, img, iters, min_inl)
    _check_against_oracle(oracle, g, obj, img, iters, min_inl)
    if noise == 0.0:
        assert g[0] and rot_angle(g[1], R.T) < 2e-6


def test_solve_pnp_edges(vsctx, oracle):
    obj, img, R, t, _ = pnp_problem(9, 0)
    assert vsctx.solve_pnp(obj, img, 100, 10)[0] is False          # n < min_inliers
    obj5, img5, _, _, _ = pnp_problem(5, 3)
    g = vsctx.solve_pnp(obj5, img5, 100, 5)                          # n == model points
    assert g[0] and g[3] == 5 and g[4].all()
    _check_against_oracle(oracle, g, obj5, img5, 100, 5)
    rng = np.random.default_rng(0)
    img_rand = np.stack([rng.uniform(0, 640, 40), rng.uniform(0, 480, 40)], 1).astype(np.float32)
    obj2, _, _, _, _ = pnp_problem(40, 1)
    g = vsctx.solve_pnp(obj2, img_rand, 100, 15)
    _check_against_oracle(oracle, g, obj2, img_rand, 100, 15)
    assert vsctx.solve_pnp(obj[:0], img[:0], 100, 10)[0] is False  # empty
    with pytest.raises(RuntimeError):
        vsctx.solve_pnp(obj2, img_rand, 4096, 15)                    # above VS_PNP_MAX_ITERS


def test_solve_pnp_batch_dev(vsctx, oracle):
    import torch
    probs = [pnp_problem(n, 100 + i, noise=0.5, outlier_frac=o) for i, (n, o) in
             enumerate([(80, 0.2), (400, 0.5), (9, 0.0), (1500, 0.3), (60, 0.6)])]
    off = np.cumsum([0] + [len(p[0]) for p in probs]).astype(np.int32)
    obj = torch.from_numpy(np.concatenate([p[0] for p in probs])).cuda()
    img = torch.from_numpy(np.concatenate([p[1] for p in probs])).cuda()
    d_off = torch.from_numpy(off).cuda()
    P = len(probs)
    dR = torch.zeros(P, 9, dtype=torch.float64, device="cuda")
    dt = torch.zeros(P, 3, dtype=torch.float64, device="cuda")
    dstat = torch.zeros(P, 8, dtype=torch.int32, device="cuda")
    dmask = torch.zeros(int(off[-1]), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    vsctx.solve_pnp_batch_dev(P, obj.data_ptr(), img.data_ptr(), d_off.data_ptr(), 300, 10, dR.data_ptr(),
                              dt.data_ptr(), dstat.data_ptr(), dmask.data_ptr())
    torch.cuda.synchronize()
    R, t, st, mask = dR.cpu().numpy(), dt.cpu().numpy(), dstat.cpu().numpy(), dmask.cpu().numpy().astype(bool)
    for p, pr in enumerate(probs):
        g = (bool(st[p, 0]), R[p].reshape(3, 3), t[p], int(st[p, 1]) if st[p, 0] else 0,
             mask[off[p]:off[p + 1]], st[p, 2:6])
        assert st[p, 6] == len(pr[0])
        _check_against_oracle(oracle, g, pr[0], pr[1], 300, 10)


def test_epnp_sequential_device_equals_host(vsctx, oracle):
    """pnp_solvers.h's sequential EPnP compiled for the device (one lane per problem; the product
    path runs the wave-parallel k_pnp_hyp, also for n == model points): the eigenvectors of
    epnp_small_eig, the pose and its Rodrigues round trip equal the host's bit for bit on 4- and
    5-point problems, noisy and exact."""
    import ctypes

    import vslam_abi
    lib = vslam_abi.load_library()
    lib.vs_debug_epnp.restype = ctypes.c_int
    lib.vs_debug_epnp.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_void_p] * 2
    rng = np.random.default_rng(9)
    count = 2000
    m = np.where(np.arange(count) % 5 == 0, 4, 5).astype(np.int32)
    X = np.zeros((count, 15))
    uv = np.zeros((count, 10))
    for p in range(count):
        obj, img, _, _, _ = pnp_problem(int(m[p]), 1000 + p, noise=0.5 if p % 2 else 0.0)
        X[p, :3 * m[p]] = obj.astype(np.float64).ravel()
        uv[p, :2 * m[p]] = img.astype(np.float64).ravel()
    K = np.array([525.0, 525.0, 319.5, 239.5])
    dev = np.zeros((count, 73))
    assert lib.vs_debug_epnp(X.ctypes.data, uv.ctypes.data, m.ctypes.data, count, K.ctypes.data, dev.ctypes.data) == 0
    host = oracle.epnp_debug(X, uv, m, tuple(K))
    bad_v = np.nonzero(np.any(dev[:, :48].view(np.uint64) != host[:, :48].view(np.uint64), axis=1))[0]
    bad_p = np.nonzero(np.any(dev[:, 48:].view(np.uint64) != host[:, 48:].view(np.uint64), axis=1))[0]
    assert len(bad_v) == 0 and len(bad_p) == 0, (bad_v[:5], bad_p[:5], np.abs(dev - host).max())
    assert host[:, 60].sum() > 0.9 * count


@pytest.mark.parametrize("mode", [1, 2])
def test_epnp_out_of_line_device_equals_host(vsctx, oracle, mode):
    """VERDICT r05 #7 regression: the sequential EPnP behind a noinline call (mode 1: one problem per lane;
    mode 2: called by lane 0 of a wave alone, as k_pnp_ransac once did) gives the host's pose and Rodrigues
    round trip bit for bit on the same 2,000 problems.  The round-5 divergence was the out-of-line code for
    B = R R^T's diagonal select (`k == a ? alpha[a] : C[k][a]`, two private arrays) reading C[k][a]
    (tools/r06/epnp_b_repro.hip); the statement now substitutes by assignment."""
    import ctypes

    import vslam_abi
    lib = vslam_abi.load_library()
    lib.vs_debug_epnp_mode.restype = ctypes.c_int
    lib.vs_debug_epnp_mode.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int]
    rng = np.random.default_rng(9)
    count = 2000
    m = np.where(np.arange(count) % 5 == 0, 4, 5).astype(np.int32)
    X = np.zeros((count, 15))
    uv = np.zeros((count, 10))
    for p in range(count):
        obj, img, _, _, _ = pnp_problem(int(m[p]), 1000 + p, noise=0.5 if p % 2 else 0.0)
        X[p, :3 * m[p]] = obj.astype(np.float64).ravel()
        uv[p, :2 * m[p]] = img.astype(np.float64).ravel()
    K = np.array([525.0, 525.0, 319.5, 239.5])
    dev = np.zeros((count, 73))
    assert lib.vs_debug_epnp_mode(X.ctypes.data, uv.ctypes.data, m.ctypes.data, count, K.ctypes.data,
                                  dev.ctypes.data, mode) == 0
    host = oracle.epnp_debug(X, uv, m, tuple(K))
    bad = np.nonzero(np.any(dev[:, 48:].view(np.uint64) != host[:, 48:].view(np.uint64), axis=1))[0]
    print("mode", mode, "differing problems:", len(bad), "max |d|", np.abs(dev[:, 48:] - host[:, 48:]).max())
    assert len(bad) == 0, (bad[:5], np.abs(dev[:, 48:] - host[:, 48:]).max())


def test_epnp_eig_stages_out_of_line(vsctx, oracle):
    """epnp_small_eig called out of line on the device dumps its stage results (QR, B = R R^T, the
    tridiagonal, the multisection brackets, the inverse iteration, v); every stage equals the host's bit
    for bit (the stage the round-5 divergence started at was B)."""
    import ctypes

    import vslam_abi
    lib = vslam_abi.load_library()
    lib.vs_debug_epnp_mode.restype = ctypes.c_int
    lib.vs_debug_epnp_mode.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int]
    count = 200
    m = np.where(np.arange(count) % 5 == 0, 4, 5).astype(np.int32)
    X = np.zeros((count, 15))
    uv = np.zeros((count, 10))
    for p in range(count):
        obj, img, _, _, _ = pnp_problem(int(m[p]), 1000 + p, noise=0.5 if p % 2 else 0.0)
        X[p, :3 * m[p]] = obj.astype(np.float64).ravel()
        uv[p, :2 * m[p]] = img.astype(np.float64).ravel()
    K = np.array([525.0, 525.0, 319.5, 239.5])
    dev = np.zeros((count, 216))
    assert lib.vs_debug_epnp_mode(X.ctypes.data, uv.ctypes.data, m.ctypes.data, count, K.ctypes.data,
                                  dev.ctypes.data, 3) == 0
    host = oracle.epnp_eig_stages(X, uv, m, tuple(K))
    stages = [("alpha", 0, 10), ("tau", 10, 20), ("B", 20, 120), ("d", 120, 130), ("e", 130, 139), ("scale", 139, 140),
              ("lo", 140, 141), ("hi", 141, 142), ("a", 142, 144), ("b", 144, 146), ("lambda", 146, 148),
              ("y", 148, 168), ("v", 168, 216)]
    total = 0
    for name, a, b in stages:
        bad = np.nonzero(np.any(dev[:, a:b].view(np.uint64) != host[:, a:b].view(np.uint64), axis=1))[0]
        print(f"stage {name:7s}: {len(bad):4d} problems differ; first {bad[:3].tolist()}",
              "" if not len(bad) else f"dev {dev[bad[0], a:min(b, a + 4)].tolist()} host {host[bad[0], a:min(b, a + 4)].tolist()}")
        total += len(bad)
    assert total == 0
