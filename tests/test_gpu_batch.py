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
