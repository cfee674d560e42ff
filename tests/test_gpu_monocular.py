"""GPU parity for the monocular 1280x720 stream (BASELINE config[4]).

The reference's monocular path is Slam::process_frame without a depth image: FeatureExtractor::extract
(FeatureExtractor.cpp:49-259) at the stream's resolution, ratio matching (Slam.cpp:1140-1172), F
verification (:880-910), and -- estimate_motion_3d3d finding no depth-valid correspondence --
Slam::estimate_motion (:1193-1213: findEssentialMat + recoverPose) with no depth scale, so the pose
chain falls back to the last good scale / MOTION_SCALE (:976-980).  Checked here at 1280x720 with
the build's HD camera (synth.K_HD): the network against the oracle's CPU network, keypoints and
descriptors bit-exact against the oracle's post-processing, and the device pipeline's per-pair
essential-matrix motion exactly equal to the oracle's estimate_motion on the same kept matches."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _kp_equal(a, b):
    return len(a) == len(b) and np.array_equal(a.view(np.uint8), b.view(np.uint8))


def _bits_equal(a, b):
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint32),
                                                 np.ascontiguousarray(b).view(np.uint32))


@pytest.fixture(scope="module")
def hd4():
    import synth
    poses = synth.loop_trajectory(126)
    out = [synth._render_one((i, R, t, synth.SEED, synth.K_HD, synth.W_HD, synth.H_HD))
           for i, (R, t) in enumerate(poses[:4])]
    return np.stack([o[0] for o in out])


def test_hd_network_matches_oracle_cpu_network(vsctx, oracle, hd4):
    gray = oracle.gray_to_f32(oracle.bgr_to_gray(hd4[0]))
    assert gray.shape == (720, 1280)
    semi, desc = vsctx.superpoint_forward(gray)
    os_, od = oracle.superpoint_forward(vsctx.weights(), gray)
    assert semi.shape == os_.shape and desc.shape == od.shape
    assert np.max(np.abs(semi - os_)) <= 2e-4 * max(1.0, float(np.max(np.abs(os_))))
    assert np.max(np.abs(desc - od)) <= 2e-5


def test_hd_extract_bit_exact(vsctx, oracle, hd4):
    feats = vsctx.extract_batch(list(hd4))
    for b in range(len(hd4)):
        gray = oracle.gray_to_f32(oracle.bgr_to_gray(hd4[b]))
        semi, dg = vsctx.superpoint_forward(gray)
        ko, do = oracle.postprocess(semi, dg, h=720, w=1280, order_mode=1)
        assert len(ko) > 0
        assert _kp_equal(feats[b][0], ko) and _bits_equal(feats[b][1], do)


def test_monocular_pipeline_matches_oracle_estimate_motion(vsctx, oracle, hd4):
    import torch

    import synth
    from vslam_pipeline import DevicePipeline, PoseChain, MOTION_SCALE
    B = len(hd4)
    pipe = DevicePipeline(vsctx, B=B, h=720, w=1280, K=synth.K_HD, monocular=True)
    frames = torch.from_numpy(hd4).cuda()
    pipe.run(frames, None, frame_count0=0)  # step 0: slot 0 of the next step = frame 3
    out = pipe.run(frames, None, frame_count0=B)
    torch.cuda.synchronize()
    feats = vsctx.extract_batch(list(hd4))
    ngood, nkept = out["ngood"].cpu().numpy(), out["nkept"].cpu().numpy()
    kept_all = out["kept"].cpu().numpy().view(np.uint8)
    assert not out["ok"].cpu().numpy().any()  # no 3D-3D stage on a monocular stream
    n_ok = 0
    for p in range(B):  # pair p = frames (p-1 mod B, p): pair 0 pairs the carried frame 3 with 0
        q = (p - 1) % B
        _, good = vsctx.match_ratio(feats[q][1], feats[p][1])
        assert ngood[p] == len(good) > 0
        k1, k2 = feats[q][0], feats[p][0]
        p1 = np.stack([k1["x"][good["query_idx"]], k1["y"][good["query_idx"]]], 1)
        p2 = np.stack([k2["x"][good["train_idx"]], k2["y"][good["train_idx"]]], 1)
        okf, F, fmask, fdiag, ferr = vsctx.find_fundamental(p1, p2)
        keep = np.flatnonzero(fmask) if okf else np.arange(len(good))
        assert nkept[p] == len(keep)
        assert np.array_equal(kept_all[p].view(good.dtype)[:nkept[p]], good[keep])
        p1, p2 = p1[keep], p2[keep]
        oko, Ro, to, mo, inl, goodo = oracle.estimate_motion(p1, p2, K=synth.K_HD)
        assert bool(out["eok"][p].item()) == oko
        assert out["escale"][p].item() == -1.0  # no depth: no scale
        if oko:
            n_ok += 1
            assert np.array_equal(out["eR"][p].cpu().numpy(), np.asarray(Ro).reshape(9))
            assert np.array_equal(out["et"][p].cpu().numpy(), np.asarray(to).reshape(3))
            assert out["ediag"][p, 3].item() == inl and out["ediag"][p, 4].item() == goodo
    assert n_ok >= 2
    # the pose chain takes MOTION_SCALE for every scale-less estimate
    chain = PoseChain()
    ok, R, t, eok, eR, et, esc = (out[k].cpu().numpy() for k in ("ok", "R", "t", "eok", "eR", "et", "escale"))
    for p in range(B):
        t0 = chain.t.copy()
        Rn, tn = chain.step(ok[p], R[p], t[p], eok[p], eR[p], et[p], esc[p])
        if eok[p]:
            assert np.isclose(np.linalg.norm(tn - t0), MOTION_SCALE * np.linalg.norm(et[p]), rtol=1e-12)
