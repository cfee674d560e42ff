"""The offline frame-sharded front end behind the C ABI (vs_batch_*, csrc/batch.hip; BASELINE
config[3]) against python/vslam_pipeline.DevicePipeline on the same frames: every
pair motion (3D-3D and E results, match counts) bit for bit, without a communicator (the carry of
the previous step's last frame) and with a one-rank RCCL communicator (the halo ring and the all-gather
exchange paths with the previous step's last depth as the halo).  More ranks need more GPUs than the
test box has; the exchange logic itself is the one the gloo tests cover for DevicePipeline."""
import numpy as np
import pytest
import torch

import synth
import vslam_abi
from vslam_pipeline import DevicePipeline

pytestmark = pytest.mark.gpu

B = 16
STEPS = 3


@pytest.fixture(scope="module")
def frames():
    L = synth.loop_sequence(126, workers=8)
    return L["bgr"][:B * STEPS], L["depth"][:B * STEPS]


@pytest.fixture(scope="module")
def pipeline_results(vsctx, frames):
    dev = torch.device("cuda", 0)
    bgr, dep = frames
    pipe = DevicePipeline(vsctx, B)
    res = []
    for k in range(STEPS):
        fr = torch.from_numpy(bgr[k * B:(k + 1) * B]).to(dev)
        de = torch.from_numpy(dep[k * B:(k + 1) * B]).to(dev)
        S = pipe.submit(fr, de, frame_count0=k * B)
        ok, R, t, eok, eR, et, esc = pipe.collect(S)
        ngood = DevicePipeline.outputs(S)["ngood"].cpu().numpy()
        res.append(dict(ok=ok, R=R, t=t, eok=eok, eR=eR, et=et, escale=esc, n_good=ngood))
    return res


@pytest.mark.parametrize("mode", ["none", "ring", "gather"])
def test_batch_c_abi_equals_device_pipeline(vsctx, frames, pipeline_results, mode):
    dev = torch.device("cuda", 0)
    bgr, dep = frames
    with_comm = mode != "none"
    uid = vslam_abi.batch_unique_id() if with_comm else None
    with vslam_abi.Batch(vsctx, B, uid=uid) as bt:
        if mode == "gather":
            bt.set_gather(True)
        if with_comm:  # a communicator needs the neighbour's depth after rank 0's first step
            with pytest.raises(vslam_abi.VSError, match="d_depth_prev"):
                fr0 = torch.from_numpy(bgr[:B]).to(dev)
                de0 = torch.from_numpy(dep[:B]).to(dev)
                bt.step_dev(fr0.data_ptr(), de0.data_ptr(), None, 0, torch.cuda.current_stream().cuda_stream)
                bt.step_dev(fr0.data_ptr(), de0.data_ptr(), None, B, torch.cuda.current_stream().cuda_stream)
    with vslam_abi.Batch(vsctx, B, uid=vslam_abi.batch_unique_id() if with_comm else None) as bt:
        if mode == "gather":
            bt.set_gather(True)
        prev = None
        for k in range(STEPS):
            fr = torch.from_numpy(bgr[k * B:(k + 1) * B]).to(dev)
            de = torch.from_numpy(dep[k * B:(k + 1) * B]).to(dev)
            torch.cuda.synchronize()
            r = bt.step_dev(fr.data_ptr(), de.data_ptr(), prev.data_ptr() if (with_comm and prev is not None) else None,
                            k * B, torch.cuda.current_stream().cuda_stream)
            prev = de[-1].clone()
            p = pipeline_results[k]
            assert np.array_equal(r["ok"], p["ok"]) and np.array_equal(r["eok"], p["eok"])
            assert np.array_equal(r["n_good"], p["n_good"])
            assert np.array_equal(r["R"].reshape(B, 9)[r["ok"] == 1], p["R"].reshape(B, 9)[p["ok"] == 1])
            assert np.array_equal(r["t"][r["ok"] == 1], p["t"][p["ok"] == 1])
            e = r["eok"] == 1
            assert np.array_equal(r["eR"].reshape(B, 9)[e], p["eR"].reshape(B, 9)[e])
            assert np.array_equal(r["escale"][e], p["escale"][e])
            assert r["ok"][1:].sum() >= B - 3  # the pairs inside the block track on this sequence


@pytest.mark.parametrize("mode", ["none", "ring"])
def test_batch_submit_collect_pipelined_equals_steps(vsctx, frames, pipeline_results, mode):
    """vs_batch_submit_dev / vs_batch_collect with two steps in flight (step k + 1's network beside step
    k's geometry, round 5) give the same pair motions as the synchronous steps; a third submit while
    two are in flight, and a collect with none, are refused."""
    dev = torch.device("cuda", 0)
    bgr, dep = frames
    with_comm = mode != "none"
    fr = [torch.from_numpy(bgr[k * B:(k + 1) * B]).to(dev) for k in range(STEPS)]
    de = [torch.from_numpy(dep[k * B:(k + 1) * B]).to(dev) for k in range(STEPS)]
    s = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    with vslam_abi.Batch(vsctx, B, uid=vslam_abi.batch_unique_id() if with_comm else None) as bt:
        with pytest.raises(vslam_abi.VSError, match="no step in flight"):
            bt.collect()
        halo = lambda k: de[k - 1][-1].data_ptr() if (with_comm and k > 0) else None
        bt.submit_dev(fr[0].data_ptr(), de[0].data_ptr(), halo(0), 0, s)
        bt.submit_dev(fr[1].data_ptr(), de[1].data_ptr(), halo(1), B, s)
        with pytest.raises(vslam_abi.VSError, match="in flight"):
            bt.submit_dev(fr[2].data_ptr(), de[2].data_ptr(), halo(2), 2 * B, s)
        out = [bt.collect()]
        bt.submit_dev(fr[2].data_ptr(), de[2].data_ptr(), halo(2), 2 * B, s)
        out += [bt.collect(), bt.collect()]
    for k in range(STEPS):
        r, p = out[k], pipeline_results[k]
        assert np.array_equal(r["ok"], p["ok"]) and np.array_equal(r["eok"], p["eok"])
        assert np.array_equal(r["n_good"], p["n_good"])
        assert np.array_equal(r["R"].reshape(B, 9)[r["ok"] == 1], p["R"].reshape(B, 9)[p["ok"] == 1])
        assert np.array_equal(r["t"][r["ok"] == 1], p["t"][p["ok"] == 1])
        e = r["eok"] == 1
        assert np.array_equal(r["eR"].reshape(B, 9)[e], p["eR"].reshape(B, 9)[e])
        assert np.array_equal(r["escale"][e], p["escale"][e])


@pytest.fixture(scope="module")
def drive_frames():
    """Distinct frames of the headline's Pioneer-like drive (every pair a new view)."""
    poses = synth.pioneer_trajectory(848)
    return synth.render_frames(poses, list(range(2 * B)), workers=8)


@pytest.mark.parametrize("mode", ["none", "ring", "gather"])
def test_batch_step_equals_oracle(vsctx, oracle, drive_frames, mode):
    """config[3]'s C ABI step against the CPU oracle directly (not through
    DevicePipeline): for every pair (frame p - 1, frame p) of a step, the oracle's ratio matching
    (Slam.cpp:1140-1172), F verification (:880-910), 3D-3D RANSAC with seed 42 + frame index (:214-375)
    and, where it fails, the E-matrix motion + depth scale (:1193-1213, :73-207) on the same GPU
    features: n_good, ok, eok exact; 3D-3D R, t <= 1e-12; E R, t, scale <= 1e-9.  Step 1's
    pair 0 joins the previous step's last frame: the carry without a communicator, the one-rank RCCL
    ring / all-gather with one."""
    dev = torch.device("cuda", 0)
    bgr, dep = drive_frames
    feats = vsctx.extract_batch(list(bgr))
    with_comm = mode != "none"
    s = torch.cuda.current_stream().cuda_stream
    out = []
    with vslam_abi.Batch(vsctx, B, uid=vslam_abi.batch_unique_id() if with_comm else None) as bt:
        if mode == "gather":
            bt.set_gather(True)
        for k in range(2):
            fr = torch.from_numpy(bgr[k * B:(k + 1) * B]).to(dev)
            de = torch.from_numpy(dep[k * B:(k + 1) * B]).to(dev)
            halo = torch.from_numpy(dep[k * B - 1]).to(dev) if (with_comm and k > 0) else None
            torch.cuda.synchronize()
            out.append(bt.step_dev(fr.data_ptr(), de.data_ptr(), None if halo is None else halo.data_ptr(), k * B, s))
    checked = n3 = nE = 0
    for k in range(2):
        r = out[k]
        for p in range(B):
            g = k * B + p
            if g == 0:
                continue  # no previous frame
            (k0, d0), (k1, d1) = feats[g - 1], feats[g]
            _, good = oracle.match_ratio(d0, d1)
            assert r["n_good"][p] == len(good), (k, p)
            _, keep, _, _ = oracle.fmat_verify(k0, k1, good)
            kept = good[keep]
            p1 = np.stack([k0["x"][kept["query_idx"]], k0["y"][kept["query_idx"]]], 1)
            p2 = np.stack([k1["x"][kept["train_idx"]], k1["y"][kept["train_idx"]]], 1)
            ok, R, t, _ = oracle.ransac_3d3d(p1, p2, dep[g - 1], dep[g], seed=42 + g)
            assert bool(r["ok"][p]) == ok, (k, p)
            if ok:
                n3 += 1
                assert np.abs(r["R"].reshape(B, 3, 3)[p] - R).max() <= 1e-12
                assert np.abs(r["t"][p] - t).max() <= 1e-12
            else:
                eok, eR, et, _, _, _ = oracle.estimate_motion(p1, p2)
                assert bool(r["eok"][p]) == eok, (k, p)
                if eok:
                    nE += 1
                    sc = oracle.estimate_scale(p1, p2, eR, et, dep[g - 1], dep[g])
                    assert np.abs(r["eR"].reshape(B, 3, 3)[p] - eR).max() <= 1e-9
                    assert np.abs(r["et"][p] - et).max() <= 1e-9 and abs(r["escale"][p] - sc) <= 1e-9
            checked += 1
    print(mode, checked, "pairs:", n3, "3D-3D,", nE, "E")
    assert checked == 2 * B - 1 and n3 >= B
