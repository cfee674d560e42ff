"""CPU tests pinning the oracle (oracle/liboracle.so) against independent restatements,
known-answer geometry and exhaustive numerics checks.  No GPU needed."""
import numpy as np
import pytest

import restate


def test_glibc_expf_restatement_exhaustive(oracle):
    # the product's device exp (glibc_expf.h) == the running libm expf for every float in [-110, 0]
    assert oracle.expf_restated_check(-110.0, 0.0, 1) == 0


def test_glibc_expf_is_not_correctly_rounded(oracle):
    # documents why glibc_expf.h exists: (float)exp((double)x) differs from glibc on ~1e-4 inputs
    assert oracle.expf_exhaustive_check(-1.0, -0.5) > 0


def test_mt19937_known_answer(oracle):
    # C++ standard [rand.predef]: the 10000th output of a default-constructed mt19937 is 4123659995
    assert int(oracle.mt19937(5489, 10000)[-1]) == 4123659995


def _mwc_steps(s, k):
    for _ in range(k):
        s = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & 0xFFFFFFFFFFFFFFFF
    return s


def test_cv_rng_jump_ahead_equals_stepping(oracle):
    """The device draws cv::RNG states out of order as s * A^k mod (A 2^32 - 1) (pnp_solvers.h);
    every jump must equal plain sequential stepping of the multiply-with-carry generator."""
    s1 = _mwc_steps(2 ** 64 - 1, 1)  # cv::RNG((uint64)-1) after its first draw
    rng = np.random.default_rng(7)
    starts = [s1, _mwc_steps(s1, 12345), 1, 2 ** 32, (4164903690 << 32) - 2]
    starts += [int(v) for v in rng.integers(1, 2 ** 62, 5)]
    for s in starts:
        for k in (0, 1, 2, 63, 64, 65, 1000, 1919, 5000):
            assert oracle.mwc_jump(s, k) == _mwc_steps(s, k), (s, k)


def _random_semi(rng, hc, wc, scale=4.0):
    return (rng.standard_normal((65, hc, wc)) * scale).astype(np.float32)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_decode_matches_numpy_restatement(oracle, seed):
    rng = np.random.default_rng(seed)
    semi = _random_semi(rng, 6, 10)
    heat_o = oracle.decode_heatmap(semi)
    heat_n = restate.decode_heatmap(semi, oracle.expf)
    assert np.array_equal(heat_o.view(np.uint32), heat_n.view(np.uint32))


def _kp_tuples(kps):
    return [(int(k["x"]), int(k["y"]), float(k["response"])) for k in kps]


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("max_kp", [400, 25])
def test_nms_oracle_matches_python_greedy(oracle, seed, max_kp):
    rng = np.random.default_rng(100 + seed)
    heat = rng.random((48, 64), dtype=np.float32) * np.float32(0.02)
    kps, ncand, _ = oracle.nms(heat, max_kp=max_kp, order_mode=1)
    ref = restate.greedy_nms(heat, max_kp=max_kp, stable=True)
    assert _kp_tuples(kps) == ref
    assert ncand == int((heat > np.float32(0.005)).sum())
    assert all(k["size"] == 8.0 and k["angle"] == -1.0 and k["octave"] == 0 and k["class_id"] == -1 for k in kps)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("max_kp", [400, 30])
def test_parallel_mis_rounds_equal_sequential_greedy(oracle, seed, max_kp):
    """The GPU NMS algorithm (priority-MIS rounds + top-K) == the reference's sorted greedy,
    including exact score ties (quantised heatmap) and the max_kp cap."""
    rng = np.random.default_rng(200 + seed)
    heat = rng.random((40, 56), dtype=np.float32) * np.float32(0.03)
    if seed % 2:
        heat = np.round(heat * 300) / 300  # many exact ties
        heat = heat.astype(np.float32)
    mis, rounds = restate.mis_rounds_nms(heat, max_kp=max_kp)
    kps, _, _ = oracle.nms(heat, max_kp=max_kp, order_mode=1)
    assert mis == _kp_tuples(kps)
    assert rounds >= 1


def _tie_heat(rng, h, w, levels, scale=0.05):
    heat = rng.random((h, w), dtype=np.float32) * np.float32(scale)
    if levels:
        heat = (np.round(heat * levels) / levels).astype(np.float32)  # exact ties
    return heat


@pytest.mark.parametrize("seed", range(10))
@pytest.mark.parametrize("max_kp", [400, 20])
def test_nms_tie_stats_oracle_matches_numpy(oracle, seed, max_kp):
    rng = np.random.default_rng(300 + seed)
    heat = _tie_heat(rng, 40, 64, [0, 60, 400, 4000][seed % 4])
    assert oracle.nms_ties(heat, max_kp=max_kp) == restate.nms_ties(heat, max_kp=max_kp)


@pytest.mark.parametrize("seed", range(24))
def test_nms_tie_free_frames_are_order_independent(oracle, seed):
    """SURVEY hard part (i): the reference's std::sort is unstable.  When a frame has no window tie
    and no cut tie, EVERY order of equal scores gives the same keypoints — the literal std::sort
    (order_mode=0) and random tie orders included; a difference needs a counted tie."""
    rng = np.random.default_rng(400 + seed)
    max_kp = [400, 25, 60][seed % 3]
    heat = _tie_heat(rng, 48, 64, [0, 40, 150, 2000][seed % 4], scale=[0.05, 0.02][seed % 2])
    window, cut, order = oracle.nms_ties(heat, max_kp=max_kp)
    stable = _kp_tuples(oracle.nms(heat, max_kp=max_kp, order_mode=1)[0])
    lit = _kp_tuples(oracle.nms(heat, max_kp=max_kp, order_mode=0)[0])
    n = int((heat > np.float32(0.005)).sum())
    others = [restate.greedy_kept(heat, order=rng.permutation(n))[:max_kp] for _ in range(4)]
    if window == 0 and cut == 0:  # the same keypoint set for every tie order
        assert sorted(lit) == sorted(stable) and all(sorted(o) == sorted(stable) for o in others)
        if order == 0:  # ... and the same list
            assert lit == stable and all(o == stable for o in others)
    elif lit != stable or any(o != stable for o in others):
        assert window + cut + order > 0


def test_nms_ties_detected_when_they_decide(oracle):
    # two equal scores side by side: which one is kept depends on the order -> a window tie
    heat = np.zeros((20, 20), np.float32)
    heat[5, 5] = heat[5, 7] = 0.5
    assert oracle.nms_ties(heat) == (1, 0, 0)
    # the 2nd and 3rd kept pixel score the same with max_kp = 2 -> a cut tie; with max_kp = 3 both
    # are output: the set is fixed, their order in the list is not -> two order ties
    heat = np.zeros((20, 40), np.float32)
    heat[2, 2], heat[2, 15], heat[2, 30] = 0.9, 0.5, 0.5
    assert oracle.nms_ties(heat, max_kp=2) == (0, 1, 0)
    assert oracle.nms_ties(heat, max_kp=3) == (0, 0, 2)


@pytest.mark.parametrize("seed", range(12))
def test_nms_score_floor_keeps_the_greedy_output(seed):
    """The GPU prunes pixels below F = the max_kp-th largest strict-local-maximum score before the
    MIS rounds (sp_post.hip): the greedy's top max_kp is unchanged, for dense and sparse heatmaps,
    with exact ties, and at caps above the number of local maxima (no floor)."""
    rng = np.random.default_rng(500 + seed)
    max_kp = [400, 30, 5, 100][seed % 4]
    heat = _tie_heat(rng, 64, 96, [0, 100, 0, 1000][seed % 4], scale=[0.03, 0.5, 0.01, 0.2][seed % 4])
    if seed >= 8:  # sparse blobs (a camera frame's shape)
        heat = np.where(rng.random(heat.shape) < 0.05, heat * 10, np.float32(0.001)).astype(np.float32)
    F = restate.nms_floor(heat, max_kp=max_kp)
    pruned = np.where(heat >= F, heat, np.float32(0)).astype(np.float32)
    assert restate.greedy_nms(pruned, max_kp=max_kp) == restate.greedy_nms(heat, max_kp=max_kp)
    if F > 0:
        assert (heat >= F).sum() < (heat > np.float32(0.005)).sum()


def test_nms_border_erase_and_empty(oracle):
    heat = np.zeros((16, 24), np.float32)
    kps, ncand, _ = oracle.nms(heat)
    assert len(kps) == 0 and ncand == 0
    heat[15, 23] = 0.5
    heat[2, 2] = 0.4
    kps, _, _ = oracle.nms(heat, h=14, w=22)  # padded image: kp at (23, 15) is erased
    assert _kp_tuples(kps) == [(2, 2, float(np.float32(0.4)))]


@pytest.mark.parametrize("seed", [0, 1])
def test_sample_matches_numpy_restatement(oracle, seed):
    rng = np.random.default_rng(seed)
    dg = rng.standard_normal((256, 6, 10)).astype(np.float32)
    xy = [(0, 0), (79, 47), (13, 5), (40, 23), (7, 46)] + [tuple(rng.integers(0, (80, 48))) for _ in range(20)]
    kps = np.zeros(len(xy), oracle.KEYPOINT_DTYPE)
    kps["x"] = [p[0] for p in xy]
    kps["y"] = [p[1] for p in xy]
    got = oracle.sample_descriptors(dg, kps)
    ref = restate.sample_descriptors(dg, xy)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def _torch_superpoint(weights, img):
    import torch
    import torch.nn.functional as F
    layers = [(1, 64, 3), (64, 64, 3), (64, 64, 3), (64, 64, 3), (64, 128, 3), (128, 128, 3), (128, 128, 3),
              (128, 128, 3), (128, 256, 3), (256, 65, 1), (128, 256, 3), (256, 256, 1)]
    ps, off = [], 0
    for cin, cout, k in layers:
        n = cout * cin * k * k
        w = torch.from_numpy(weights[off:off + n].reshape(cout, cin, k, k).astype(np.float64))
        off += n
        b = torch.from_numpy(weights[off:off + cout].astype(np.float64))
        off += cout
        ps.append((w, b, k // 2))
    x = torch.from_numpy(img.astype(np.float64))[None, None]
    c = lambda x, i: F.conv2d(x, ps[i][0], ps[i][1], padding=ps[i][2])
    x = F.relu(c(x, 0)); x = F.relu(c(x, 1)); x = F.max_pool2d(x, 2)
    x = F.relu(c(x, 2)); x = F.relu(c(x, 3)); x = F.max_pool2d(x, 2)
    x = F.relu(c(x, 4)); x = F.relu(c(x, 5)); x = F.max_pool2d(x, 2)
    x = F.relu(c(x, 6)); x = F.relu(c(x, 7))
    semi = c(F.relu(c(x, 8)), 9)
    desc = c(F.relu(c(x, 10)), 11)
    desc = desc / torch.norm(desc, p=2, dim=1, keepdim=True)
    return semi[0].numpy(), desc[0].numpy()


def synthetic_weights(seed=5):
    rng = np.random.default_rng(seed)
    layers = [(1, 64, 3), (64, 64, 3), (64, 64, 3), (64, 64, 3), (64, 128, 3), (128, 128, 3), (128, 128, 3),
              (128, 128, 3), (128, 256, 3), (256, 65, 1), (128, 256, 3), (256, 256, 1)]
    parts = []
    for cin, cout, k in layers:
        parts.append(rng.standard_normal(cout * cin * k * k) * np.sqrt(2.0 / (cin * k * k)))
        parts.append(rng.standard_normal(cout) * 0.05)
    return np.concatenate(parts).astype(np.float32)


def test_oracle_superpoint_matches_torch_fp64(oracle):
    w = synthetic_weights()
    assert w.size == oracle.lib().orc_superpoint_num_params() == 1300865
    rng = np.random.default_rng(3)
    img = rng.random((64, 96), dtype=np.float32)
    semi, desc = oracle.superpoint_forward(w, img, nthreads=4)
    ts, td = _torch_superpoint(w, img)
    assert np.max(np.abs(semi - ts)) <= 1e-4 * max(1.0, np.max(np.abs(ts)))
    assert np.max(np.abs(desc - td)) <= 1e-5


def test_oracle_match_fp32_semantics_vs_fp64(oracle):
    import synth
    d1 = synth.random_descriptors(300, 1)
    d2 = np.concatenate([d1[:150] + 0.05 * synth.random_descriptors(150, 2), synth.random_descriptors(250, 3)])
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    raw32, good32 = oracle.match_ratio(d1, d2)
    raw64, good64 = oracle.match_ratio(d1, d2, f64=True)
    assert len(raw32) == len(raw64) == 300
    assert np.array_equal(raw32["train_idx"], raw64["train_idx"])
    assert np.array_equal(good32["query_idx"], good64["query_idx"])
    # the dot-product form cancels for near neighbours: bound the error on d^2, not d
    d32 = raw32["distance"].astype(np.float64) ** 2
    d64 = raw64["distance"].astype(np.float64) ** 2
    assert np.max(np.abs(d32 - d64)) < 2e-6
    # first 150 queries have a planted neighbour
    assert np.array_equal(raw32["train_idx"][:150], np.arange(150))


def test_oracle_match_edges(oracle):
    import synth
    d = synth.random_descriptors(10, 4)
    assert [len(x) for x in oracle.match_ratio(d, d[:1])] == [0, 0]   # fewer than 2 neighbours
    assert [len(x) for x in oracle.match_ratio(d[:0], d)] == [0, 0]   # empty query
    raw, good = oracle.match_ratio(d, np.concatenate([d, d]))        # exact duplicates: tie -> lower index
    assert np.array_equal(raw["train_idx"], np.arange(10))
    assert len(good) == 0  # d0 == d1 == 0 fails the strict ratio test


@pytest.mark.parametrize("seed,outliers,noise", [(0, 0.4, 0.0), (1, 0.4, 0.002), (2, 0.2, 0.001)])
def test_oracle_ransac_3d3d_known_answer(oracle, seed, outliers, noise):
    p1, p2, d1, d2, R, t, inl = restate.rigid_scene(200, outliers, seed, noise=noise)
    ok, Re, te, diag = oracle.ransac_3d3d(p1, p2, d1, d2, seed=42 + seed)
    assert ok
    tol = 1e-5 if noise == 0 else 5e-3
    assert np.max(np.abs(Re - R)) < tol and np.max(np.abs(te - t)) < tol
    assert diag[0] == 200 and diag[3] >= inl.sum() - (0 if noise == 0 else 3)
    assert abs(np.linalg.det(Re) - 1) < 1e-12


def test_oracle_ransac_3d3d_failures(oracle):
    p1, p2, d1, d2, R, t, inl = restate.rigid_scene(30, 0.0, 9)
    ok, _, _, diag = oracle.ransac_3d3d(p1[:9], p2[:9], d1, d2)
    assert not ok and diag[0] == 9  # N < 10
    z = np.zeros_like(d1)
    ok, _, _, diag = oracle.ransac_3d3d(p1, p2, z, d2)
    assert not ok and diag[0] == 0  # no valid depth
    # translation above RANSAC_3D3D_MAX_TRANSLATION (0.2 m) is rejected after the refit
    p1, p2, d1, d2, R, t, inl = restate.rigid_scene(60, 0.0, 10, trans=(0.3, 0.0, 0.0))
    ok, _, te, diag = oracle.ransac_3d3d(p1, p2, d1, d2)
    assert not ok and diag[3] == 60 and np.allclose(te, t, atol=1e-5)


def test_nms_score_floor_full_frame_dense():
    # a random-weight SuperPoint heatmap's shape: nearly every pixel a candidate, ~1/81 of them
    # strict local maxima; the floor leaves a small fraction of the candidates undecided
    rng = np.random.default_rng(77)
    heat = (rng.random((240, 320), dtype=np.float32) * np.float32(0.03)).astype(np.float32)
    F = restate.nms_floor(heat)
    assert F > 0 and (heat >= F).sum() < 0.05 * (heat > np.float32(0.005)).sum()
    pruned = np.where(heat >= F, heat, np.float32(0)).astype(np.float32)
    assert restate.greedy_nms(pruned) == restate.greedy_nms(heat)


@pytest.mark.parametrize("n1,n2,seed", [(400, 400, 1), (37, 513, 2), (1, 2, 3), (300, 33, 4)])
def test_oracle_vector_matcher_equals_scalar(oracle, n1, n2, seed):
    """The AVX2 path of orc_match_ratio (eight fmaf chains per register) == the scalar fmaf loops
    bit for bit, including planted near-duplicates and exact ties."""
    import synth
    d1 = synth.random_descriptors(n1, seed)
    d2 = synth.random_descriptors(n2, seed + 100)
    k = min(n1, n2) // 2
    d2[:k] = d1[:k] + 0.01 * synth.random_descriptors(k, seed + 200)
    if n2 > 3:
        d2[-1] = d2[0]  # an exact duplicate train row: the lower index wins
    a = oracle.match_ratio(d1, d2)
    b = oracle.match_ratio(d1, d2, scalar=True)
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8))
