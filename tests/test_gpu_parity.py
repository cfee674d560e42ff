"""GPU parity tests: libvslam_hip.so (HIP, gfx950) against the CPU oracle on identical inputs.

Bars (DESIGN.md "Parity"): keypoint pixel indices, scores, sampled descriptors and match pair
lists bit-exact; 3D-3D RANSAC decisions (ok, N, best inliers, best iteration, refit inliers)
exact and R, t within 1e-12; network outputs within the fp32 tolerance stated in each test.
"""
import numpy as np
import pytest

import restate

pytestmark = pytest.mark.gpu


def _kp_equal(a, b):
    return len(a) == len(b) and np.array_equal(a.view(np.uint8), b.view(np.uint8))


def _bits_equal(a, b):
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint32),
                                                 np.ascontiguousarray(b).view(np.uint32))


# ---------------------------------------------------------------------------------- network
def test_network_matches_torch_fp64(vsctx, seq4):
    from test_oracle import _torch_superpoint
    import oracle_py
    w = vsctx.weights()
    gray = oracle_py.gray_to_f32(oracle_py.bgr_to_gray(seq4[0]["bgr"]))
    semi, desc = vsctx.superpoint_forward(gray)
    ts, td = _torch_superpoint(w, gray)
    # fp32 accumulation over K <= 4608 products vs an fp64 reference
    tol_semi = 2e-4 * max(1.0, float(np.max(np.abs(ts))))
    assert np.max(np.abs(semi - ts)) <= tol_semi
    assert np.max(np.abs(desc - td)) <= 2e-5


@pytest.mark.parametrize("h,w", [(152, 200), (64, 96)])
def test_network_other_geometries_match_torch_fp64(vsctx, h, w):
    """Widths that are not multiples of 32 at every level: partial 8 x 32 tiles (conv1, pooled
    layers) and the raster-order linear tiles (unpooled layers at W = 100, 50, 25 / 48, 24, 12)."""
    from test_oracle import _torch_superpoint
    rng = np.random.default_rng(h * w)
    gray = rng.random((h, w), dtype=np.float32)
    semi, desc = vsctx.superpoint_forward(gray)
    ts, td = _torch_superpoint(vsctx.weights(), gray)
    assert semi.shape == ts.shape and desc.shape == td.shape
    assert np.max(np.abs(semi - ts)) <= 2e-4 * max(1.0, float(np.max(np.abs(ts))))
    assert np.max(np.abs(desc - td)) <= 2e-5


def test_network_matches_oracle_cpu_network(vsctx, oracle, seq4):
    w = vsctx.weights()
    gray = oracle.gray_to_f32(oracle.bgr_to_gray(seq4[1]["bgr"]))
    semi, desc = vsctx.superpoint_forward(gray)
    os_, od = oracle.superpoint_forward(w, gray)
    assert np.max(np.abs(semi - os_)) <= 2e-4 * max(1.0, float(np.max(np.abs(os_))))
    assert np.max(np.abs(desc - od)) <= 2e-5


# ------------------------------------------------------------------- post-processing (A4-A6)
@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_postprocess_bit_exact_random(vsctx, oracle, seed):
    rng = np.random.default_rng(seed)
    hc, wc = 60, 80
    semi = (rng.standard_normal((65, hc, wc)) * (2.0 + seed)).astype(np.float32)
    if seed == 3:  # quantised logits -> many exactly tied scores
        semi = np.round(semi * 4) / 4
    dg = rng.standard_normal((256, hc, wc)).astype(np.float32)
    dg /= np.linalg.norm(dg, axis=0, keepdims=True)
    kg, dgpu = vsctx.postprocess(semi, dg)
    ko, do = oracle.postprocess(semi, dg, order_mode=1)
    assert _kp_equal(kg, ko)
    assert _bits_equal(dgpu, do)


def test_postprocess_bit_exact_network_outputs(vsctx, oracle, seq4):
    for f in seq4:
        gray = oracle.gray_to_f32(oracle.bgr_to_gray(f["bgr"]))
        semi, dg = vsctx.superpoint_forward(gray)
        kg, dgpu = vsctx.postprocess(semi, dg)
        ko, do = oracle.postprocess(semi, dg, order_mode=1)
        assert _kp_equal(kg, ko) and _bits_equal(dgpu, do)
        assert len(kg) == 400


def test_postprocess_edges(vsctx, oracle):
    hc, wc = 12, 16
    dg = np.ones((256, hc, wc), np.float32) / 16.0
    semi = np.zeros((65, hc, wc), np.float32)
    semi[64] = 50.0  # everything in the dustbin: no candidates
    kg, d = vsctx.postprocess(semi, dg)
    assert len(kg) == 0
    # padded frame: border erase (h, w not multiples of 8), and a tiny cap
    rng = np.random.default_rng(11)
    semi = (rng.standard_normal((65, hc, wc)) * 3).astype(np.float32)
    for h, w, cap in [(93, 121, 400), (96, 128, 7), (90, 128, 1)]:
        kg, dgpu = vsctx.postprocess(semi, dg, h=h, w=w, cap=cap)
        ko, do = oracle.postprocess(semi, dg, h=h, w=w, max_kp=min(cap, 400), order_mode=1)
        assert _kp_equal(kg, ko) and _bits_equal(dgpu, do)


@pytest.mark.parametrize("hc,wc", [(19, 25), (13, 7), (5, 41)])
def test_postprocess_partial_tiles(vsctx, oracle, hc, wc):
    """Cell grids whose pixel sizes are not multiples of the 32-pixel NMS tile: the decode fused into
    k_nms_lmax (halo cells past the grid, partial tiles, the interior heatmap stores) and the
    XCD-aware tile order, bit-exact against the CPU restatement."""
    rng = np.random.default_rng(hc * 100 + wc)
    semi = (rng.standard_normal((65, hc, wc)) * 3).astype(np.float32)
    dg = rng.standard_normal((256, hc, wc)).astype(np.float32)
    dg /= np.linalg.norm(dg, axis=0, keepdims=True)
    for h, w in [(hc * 8, wc * 8), (hc * 8 - 3, wc * 8 - 5)]:
        kg, dgpu = vsctx.postprocess(semi, dg, h=h, w=w)
        ko, do = oracle.postprocess(semi, dg, h=h, w=w, order_mode=1)
        assert _kp_equal(kg, ko) and _bits_equal(dgpu, do)


def test_extract_odd_geometry_raw_grid_equals_network_plus_oracle_post(vsctx, oracle):
    """Extraction at 152 x 200 (partial NMS tiles) through the raw-grid path — the network leaves the
    descriptor grid unnormalised and the sampler normalises the corners it reads — equals the
    normalised network output post-processed by the CPU restatement, bit for bit."""
    rng = np.random.default_rng(5)
    h, w = 152, 200
    img = (rng.random((h, w, 3)) * 255).astype(np.uint8)
    img[40:90, 60:150] = 255 - img[40:90, 60:150]  # some structure
    kps, desc = vsctx.extract(img)
    gray = oracle.gray_to_f32(oracle.bgr_to_gray(img))
    semi, dg = vsctx.superpoint_forward(gray)
    ko, do = oracle.postprocess(semi, dg, h=h, w=w, order_mode=1)
    assert len(kps) > 0
    assert _kp_equal(kps, ko) and _bits_equal(desc, do)


def test_extract_end_to_end_equals_network_plus_oracle_post(vsctx, oracle, seq4):
    f = seq4[2]
    kps, desc = vsctx.extract(f["bgr"])
    gray = oracle.gray_to_f32(oracle.bgr_to_gray(f["bgr"]))
    semi, dg = vsctx.superpoint_forward(gray)
    ko, do = oracle.postprocess(semi, dg, order_mode=1)
    assert _kp_equal(kps, ko) and _bits_equal(desc, do)


def test_extract_gray_input_and_batch_consistency(vsctx, oracle, seq4):
    imgs = [f["bgr"] for f in seq4]
    batch = vsctx.extract_batch(imgs)
    for img, (kb, db) in zip(imgs, batch):
        ks, ds = vsctx.extract(img)
        assert _kp_equal(kb, ks) and _bits_equal(db, ds)
    g = oracle.bgr_to_gray(imgs[0])
    kg, dg = vsctx.extract(g)  # channels == 1 path
    assert _kp_equal(kg, batch[0][0]) and _bits_equal(dg, batch[0][1])


# ----------------------------------------------------------------------------- matching (A7)
def _match_equal(a, b):
    return len(a) == len(b) and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("n1,n2", [(400, 400), (37, 513), (1, 2), (128, 129), (300, 1000), (513, 64)])
def test_match_bit_exact_random(vsctx, oracle, n1, n2):
    import synth
    d1 = synth.random_descriptors(n1, n1 * 7 + 1)
    d2 = synth.random_descriptors(n2, n2 * 11 + 2)
    k = min(n1, n2) // 2
    d2[:k] = d1[:k] + 0.1 * synth.random_descriptors(k, 5)[:k]  # planted neighbours
    raw_g, good_g = vsctx.match_ratio(d1, d2)
    raw_o, good_o = oracle.match_ratio(d1, d2)
    assert _match_equal(raw_g, raw_o) and _match_equal(good_g, good_o)


def test_match_edges_and_ties(vsctx, oracle):
    import synth
    d = synth.random_descriptors(50, 3)
    for d1, d2 in [(d, d[:1]), (d[:0], d), (d, d[:0]), (d, np.concatenate([d, d])), (d[:1], d[:2])]:
        rg, gg = vsctx.match_ratio(d1, d2)
        ro, go = oracle.match_ratio(d1, d2)
        assert _match_equal(rg, ro) and _match_equal(gg, go)


@pytest.mark.parametrize("P", [3, 40])
def test_match_pairs_batched_bit_exact(vsctx, oracle, P):
    """One vs_match_pairs_dev launch over P pairs of a frame pool, ragged counts incl. empty /
    single-row frames and a frame paired with itself; every pair's lists must equal the oracle's.
    Run after other tests have sized the context's key state for fewer pairs, P = 40 also covers
    the state's growth (a regrown buffer may come back at the same address, uninitialised)."""
    import synth
    import torch
    cap = 400
    F = P + 2
    rng = np.random.default_rng(P)
    n = rng.integers(300, cap + 1, F).astype(np.int32)
    n[1], n[2], n[3] = 0, 1, 2
    desc = np.zeros((F, cap, 256), np.float32)
    for f in range(F):
        desc[f, :n[f]] = synth.random_descriptors(int(n[f]), 100 + f)
        if f and n[f] > 50 and n[f - 1] > 50:  # planted neighbours of the previous frame
            desc[f, :50] = desc[f - 1, :50] + 0.1 * synth.random_descriptors(50, 900 + f)
    pairs = [(f, f + 1) for f in range(P)]
    pairs[-1] = (F - 1, F - 1)
    pairs = np.array(pairs, np.int32)
    dev = torch.device("cuda", 0)
    d_desc = torch.from_numpy(desc).to(dev)
    d_n = torch.from_numpy(n).to(dev)
    d_pairs = torch.from_numpy(pairs).to(dev)
    raw = torch.zeros((P, cap, 4), dtype=torch.int32, device=dev)
    good = torch.zeros_like(raw)
    nraw = torch.full((P,), -1, dtype=torch.int32, device=dev)
    ngood = torch.full((P,), -1, dtype=torch.int32, device=dev)
    for rep in range(2):  # the second launch reuses the keys / counters the first left reset
        torch.cuda.synchronize()
        vsctx.match_pairs_dev(P, d_pairs.data_ptr(), F, d_desc.data_ptr(), d_n.data_ptr(), cap, 0.75,
                              raw.data_ptr(), nraw.data_ptr(), good.data_ptr(), ngood.data_ptr())
        torch.cuda.synchronize()
        rh, gh = raw.cpu().numpy(), good.cpu().numpy()
        nr, ng = nraw.cpu().numpy(), ngood.cpu().numpy()
        for p, (a, b) in enumerate(pairs):
            ro, go = oracle.match_ratio(desc[a, :n[a]], desc[b, :n[b]])
            assert nr[p] == len(ro) and ng[p] == len(go), (p, nr[p], len(ro), ng[p], len(go))
            assert np.array_equal(rh[p, :nr[p]].view(np.uint8).ravel(), ro.view(np.uint8).ravel()), p
            assert np.array_equal(gh[p, :ng[p]].view(np.uint8).ravel(), go.view(np.uint8).ravel()), p


def test_match_bit_exact_real_descriptors(vsctx, oracle, seq4):
    feats = vsctx.extract_batch([f["bgr"] for f in seq4])
    for i in range(3):
        rg, gg = vsctx.match_ratio(feats[i][1], feats[i + 1][1])
        ro, go = oracle.match_ratio(feats[i][1], feats[i + 1][1])
        assert _match_equal(rg, ro) and _match_equal(gg, go)
        assert len(gg) > 50  # consecutive synthetic frames do match


# ------------------------------------------------------------------------ 3D-3D RANSAC (A9)
def _ransac_equal(g, o):
    okg, Rg, tg, dg = g
    oko, Ro, to, do = o
    assert okg == oko
    assert np.array_equal(dg, do)
    if do[3] > 0:
        assert np.max(np.abs(Rg - Ro)) <= 1e-12 and np.max(np.abs(tg - to)) <= 1e-12


@pytest.mark.parametrize("seed,outliers,noise,n", [(0, 0.4, 0.0, 200), (1, 0.4, 0.002, 300), (2, 0.6, 0.001, 400),
                                                   (3, 0.0, 0.0, 10), (4, 0.9, 0.0, 120)])
def test_ransac_3d3d_matches_oracle(vsctx, oracle, seed, outliers, noise, n):
    p1, p2, d1, d2, R, t, inl = restate.rigid_scene(n, outliers, seed, noise=noise)
    g = vsctx.ransac_3d3d(p1, p2, d1, d2, seed=42 + seed)
    o = oracle.ransac_3d3d(p1, p2, d1, d2, seed=42 + seed)
    _ransac_equal(g, o)


def test_ransac_3d3d_on_pipeline_matches(vsctx, oracle, seq4):
    feats = vsctx.extract_batch([f["bgr"] for f in seq4])
    for i in range(3):
        (k1, d1), (k2, d2) = feats[i], feats[i + 1]
        _, good = vsctx.match_ratio(d1, d2)
        p1 = np.stack([k1["x"][good["query_idx"]], k1["y"][good["query_idx"]]], 1)
        p2 = np.stack([k2["x"][good["train_idx"]], k2["y"][good["train_idx"]]], 1)
        g = vsctx.ransac_3d3d(p1, p2, seq4[i]["depth"], seq4[i + 1]["depth"], seed=42 + i)
        o = oracle.ransac_3d3d(p1, p2, seq4[i]["depth"], seq4[i + 1]["depth"], seed=42 + i)
        _ransac_equal(g, o)


def test_ransac_3d3d_small_n_and_many_draws(vsctx, oracle):
    # N == 10 forces many rejection draws; iters = 1024 consumes > 1248 MT outputs (lane-0 twist path)
    p1, p2, d1, d2, R, t, inl = restate.rigid_scene(10, 0.3, 21)
    for iters in (200, 1024):
        g = vsctx.ransac_3d3d(p1, p2, d1, d2, seed=7, iters=iters)
        o = oracle.ransac_3d3d(p1, p2, d1, d2, seed=7, iters=iters)
        _ransac_equal(g, o)


# ------------------------------------------------------------ device-batched entry points
def test_device_pipeline_matches_host_entry_points(vsctx, seq4):
    import torch
    from vslam_pipeline import DevicePipeline
    pipe = DevicePipeline(vsctx, B=len(seq4), h=480, w=640)
    frames = torch.from_numpy(np.stack([f["bgr"] for f in seq4])).cuda()
    depth = torch.from_numpy(np.stack([f["depth"] for f in seq4])).cuda()
    out = pipe.run(frames, depth, frame_count0=0)
    torch.cuda.synchronize()
    feats = vsctx.extract_batch([f["bgr"] for f in seq4])
    n = out["n"].cpu().numpy()
    kps = out["kps"].cpu().numpy().view(np.uint8)
    for b in range(len(seq4)):
        kb = kps[b].view(feats[b][0].dtype)[:n[b]]
        assert _kp_equal(kb, feats[b][0])
    ngood = out["ngood"].cpu().numpy()
    nkept = out["nkept"].cpu().numpy()
    kept_all = out["kept"].cpu().numpy().view(np.uint8)
    assert ngood[0] == 0  # no frame before the first batch
    for p in range(1, len(seq4)):  # pair p = frames (p-1, p), seed 42 + frame_count
        _, good = vsctx.match_ratio(feats[p - 1][1], feats[p][1])
        assert ngood[p] == len(good)
        okp = bool(out["ok"][p].item())
        k1, k2 = feats[p - 1][0], feats[p][0]
        p1 = np.stack([k1["x"][good["query_idx"]], k1["y"][good["query_idx"]]], 1)
        p2 = np.stack([k2["x"][good["train_idx"]], k2["y"][good["train_idx"]]], 1)
        # F verification (Slam.cpp:880-910) filters the matches before the 3D-3D stage
        okf, F, fmask, fdiag, ferr = vsctx.find_fundamental(p1, p2)
        assert np.allclose(out["eperr"][p].cpu().numpy(), ferr, rtol=1e-12, atol=0)
        keep = np.flatnonzero(fmask) if okf else np.arange(len(good))
        assert nkept[p] == len(keep)
        assert np.array_equal(kept_all[p].view(good.dtype)[:nkept[p]], good[keep])
        assert np.array_equal(out["fdiag"][p].cpu().numpy()[:4], fdiag)
        p1, p2 = p1[keep], p2[keep]
        okh, Rh, th, dh = vsctx.ransac_3d3d(p1, p2, seq4[p - 1]["depth"], seq4[p]["depth"], seed=42 + p)
        assert okp == okh
        assert np.array_equal(out["diag"][p].cpu().numpy(), dh)
        if okh:
            assert np.max(np.abs(out["R"][p].cpu().numpy() - Rh.reshape(9))) <= 1e-12
            assert out["eok"][p].item() == 0 and out["ediag"][p, 5].item() == 0  # fallback skipped
        else:  # Slam.cpp:965-984: the essential-matrix fallback with depth scale
            oke, Re, te, sce, de = vsctx.estimate_motion(p1, p2, seq4[p - 1]["depth"], seq4[p]["depth"])
            assert bool(out["eok"][p].item()) == oke
            if oke:
                assert np.array_equal(out["eR"][p].cpu().numpy(), Re.reshape(9))
                assert np.array_equal(out["et"][p].cpu().numpy(), te) and out["escale"][p].item() == sce


def test_device_pipeline_overlapped_steps_match_synchronous(vsctx, seq4):
    """Three steps submitted back to back on the two-stream pipeline (geometry of step k beside the
    network of step k+1, buffer sets reused) give the same per-pair motion as three synchronous
    runs, including the carried halo frame between steps."""
    import torch
    from vslam_pipeline import DevicePipeline
    B = len(seq4)
    frames = torch.from_numpy(np.stack([f["bgr"] for f in seq4])).cuda()
    depth = torch.from_numpy(np.stack([f["depth"] for f in seq4])).cuda()
    sync = DevicePipeline(vsctx, B=B, h=480, w=640)
    ref = []
    for i in range(3):
        out = sync.run(frames, depth, frame_count0=i * B)
        ref.append((out["ok"].cpu().numpy(), out["R"].cpu().numpy(), out["eok"].cpu().numpy(),
                    out["eR"].cpu().numpy(), out["escale"].cpu().numpy(), out["ngood"].cpu().numpy()))
    pipe = DevicePipeline(vsctx, B=B, h=480, w=640)
    handles = [pipe.submit(frames, depth, frame_count0=i * B) for i in range(2)]
    got = [pipe.collect(handles[0])]
    handles.append(pipe.submit(frames, depth, frame_count0=2 * B))
    got += [pipe.collect(handles[1]), pipe.collect(handles[2])]
    for i in range(3):
        ok, R, t, eok, eR, et, esc = got[i]
        rok, rR, reok, reR, resc, rngood = ref[i]
        assert np.array_equal(ok, rok) and np.array_equal(R, rR)
        assert np.array_equal(eok, reok) and np.array_equal(eR, reR) and np.array_equal(esc, resc)
    assert ref[1][5][0] > 0  # the carried frame pairs with the next step's first frame


def test_profile_reports_stages(vsctx, seq4):
    vsctx.profile(True)
    vsctx.profile_reset()
    vsctx.extract(seq4[0]["bgr"])
    prof = vsctx.profile_read()
    vsctx.profile(False)
    for st in ["conv1_fused", "conv2a", "head_a", "nms_rounds", "sample"]:
        assert st in prof and prof[st][0] > 0


# --------------------------------------------- NMS beyond the tile-round budget
def _unit_grid(hc, wc, seed):
    dg = np.random.default_rng(seed).standard_normal((256, hc, wc)).astype(np.float32)
    return dg / np.linalg.norm(dg, axis=0, keepdims=True)


@pytest.mark.parametrize("case", ["serpentine", "gradient"])
def test_postprocess_long_dependency_chains(vsctx, oracle, case):
    """Heatmaps the 8 tile rounds cannot settle (tests/nms_cases.py: a ~4900-pixel chain through
    every tile, thousands of priority-MIS rounds; a whole-frame score gradient): k_nms_finish
    completes them and the keypoints equal the oracle's sequential greedy NMS bit for bit."""
    import nms_cases
    hc, wc = 60, 80
    semi = nms_cases.serpentine_semi(hc, wc)[0] if case == "serpentine" else nms_cases.gradient_semi(hc, wc)
    dg = _unit_grid(hc, wc, 5)
    kg, dgpu = vsctx.postprocess(semi, dg)
    ko, do = oracle.postprocess(semi, dg, order_mode=1)
    assert _kp_equal(kg, ko) and _bits_equal(dgpu, do)
    assert len(kg) == 400
    if case == "serpentine":  # the top of the chain: every other pixel, 8 apart, along row 2
        assert np.array_equal(kg["x"][:80], np.arange(0, 640, 8)) and np.all(kg["y"][:80] == 2)


def test_postprocess_round_cap_is_reported(vsctx, monkeypatch):
    """A frame that reaches k_nms_finish's round cap is an error, never a silent keypoint list:
    VS_ERR_NOTCONV from the host entry point, d_n[b] = VS_ERR_NOTCONV (no keypoints) for that
    frame alone on the enqueue-only device path.  The cap is lowered to 2 rounds here
    (VS_NMS_FINISH_ROUNDS, a test knob) so the serpentine chain reaches it."""
    import torch
    import nms_cases
    import vslam_abi
    hc, wc = 60, 80
    semi_s, _ = nms_cases.serpentine_semi(hc, wc)
    rng = np.random.default_rng(3)
    semi_r = (rng.standard_normal((65, hc, wc)) * 3).astype(np.float32)
    dg = _unit_grid(hc, wc, 6)
    monkeypatch.setenv("VS_NMS_FINISH_ROUNDS", "2")
    with pytest.raises(vslam_abi.VSError, match="NOTCONV"):
        vsctx.postprocess(semi_s, dg)
    dev = torch.device("cuda", 0)
    semi = torch.from_numpy(np.stack([semi_s, semi_r]).transpose(0, 2, 3, 1).copy()).to(dev)
    grid = torch.from_numpy(np.stack([dg, dg]).transpose(0, 2, 3, 1).copy()).to(dev)
    cap = 400
    kps = torch.zeros((2, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((2, cap, 256), dtype=torch.float32, device=dev)
    n = torch.full((2,), 12345, dtype=torch.int32, device=dev)
    vsctx.postprocess_batch_dev(2, semi.data_ptr(), grid.data_ptr(), hc * 8, wc * 8, kps.data_ptr(),
                                desc.data_ptr(), n.data_ptr(), cap)
    torch.cuda.synchronize()
    assert n.tolist() == [vslam_abi.VS_ERR_NOTCONV, 400]
    monkeypatch.delenv("VS_NMS_FINISH_ROUNDS")
    kg, _ = vsctx.postprocess(semi_r, dg)
    assert np.array_equal(kps[1].cpu().numpy().view(np.uint8).reshape(-1)[:kg.nbytes], kg.view(np.uint8).reshape(-1))


# ------------------------------------------ NMS ties vs the reference's std::sort
def _tie_delta(ctx, before):
    after = ctx.tie_stats()
    return tuple(after[k] - before[k] for k in ("window_ties", "cut_ties", "order_ties"))


def test_nms_tie_counts_and_literal_std_sort(vsctx, oracle):
    """SURVEY hard part (i).  For camera frames of the synthetic sequence and for tie-heavy
    (quantised) heatmaps: the GPU's per-frame tie counts equal the oracle's (orc_nms_ties), and the
    GPU keypoints are compared with the literal std::sort path of the oracle (order_mode=0, the
    reference's unstable sort under libstdc++).  A frame whose keypoints differ from std::sort's
    must carry a counted tie; the mismatch and tie counts are recorded in
    gpurun_out/nms_literal_sort.json."""
    import json
    import os

    import synth
    seq = synth.loop_sequence(24, workers=8)
    cases = [("camera", oracle.gray_to_f32(oracle.bgr_to_gray(img))) for img in seq["bgr"]]
    rng = np.random.default_rng(21)
    for q in (1, 2, 4):  # coarse logits, flat cells: many exactly equal scores among candidates
        semi = np.round(rng.standard_normal((65, 60, 80)).astype(np.float32) * 0.5 * q) / q
        cases.append((f"quantised/{q}", semi.astype(np.float32)))
    dg_q = _unit_grid(60, 80, 9)
    rec = {"frames": 0, "mismatch_vs_std_sort": 0, "set_mismatch_vs_std_sort": 0, "frames_with_tie": 0,
           "window_ties": 0, "cut_ties": 0, "order_ties": 0, "mismatch_without_tie": 0,
           "set_mismatch_without_set_tie": 0, "by_kind": {}}
    for kind, x in cases:
        if kind == "camera":
            semi, dg = vsctx.superpoint_forward(x)
        else:
            semi, dg = x, dg_q
        before = vsctx.tie_stats()
        kg, _ = vsctx.postprocess(semi, dg)
        w, c, o = _tie_delta(vsctx, before)
        assert (w, c, o) == oracle.nms_ties(oracle.decode_heatmap(semi)), kind
        ko_stable, _ = oracle.postprocess(semi, dg, order_mode=1)
        assert _kp_equal(kg, ko_stable)
        ko_lit, _ = oracle.postprocess(semi, dg, order_mode=0)
        differ = not _kp_equal(kg, ko_lit)
        key = lambda k: sorted(zip(k["x"].tolist(), k["y"].tolist()))
        set_differ = key(kg) != key(ko_lit)
        rec["frames"] += 1
        rec["mismatch_vs_std_sort"] += differ
        rec["set_mismatch_vs_std_sort"] += set_differ
        rec["frames_with_tie"] += (w + c + o) > 0
        rec["window_ties"] += w
        rec["cut_ties"] += c
        rec["order_ties"] += o
        rec["mismatch_without_tie"] += differ and (w + c + o) == 0
        rec["set_mismatch_without_set_tie"] += set_differ and (w + c) == 0
        k = rec["by_kind"].setdefault(kind.split("/")[0], {"frames": 0, "mismatch": 0, "tie_frames": 0})
        k["frames"] += 1
        k["mismatch"] += differ
        k["tie_frames"] += (w + c + o) > 0
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "nms_literal_sort.json"), "w") as fh:
        json.dump(rec, fh, indent=1)
    print("nms literal std::sort:", rec)
    assert rec["mismatch_without_tie"] == 0 and rec["set_mismatch_without_set_tie"] == 0
    assert rec["by_kind"]["quantised"]["tie_frames"] > 0  # the tie path is exercised
