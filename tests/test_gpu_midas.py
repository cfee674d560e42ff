"""MiDaS v2.1-small on the GPU (F3, BASELINE config[4]; reference src/DepthEstimator.cpp:39-112)
against the CPU restatements in tests/midas_ref.py.

Bars: pre-processing (8-bit resize, 1/255, per-plane normalisation) bit-exact; the network
(fp32 MFMA implicit GEMMs, fp32 depthwise / bilinear) within 1e-4 of the output's range against
torch float64 on the same weights and input (stated per test); post-processing (float resize,
min-max) within 2e-6 absolute on the [0, 1] map; the device pipeline equals its three stages
chained and is batch-independent bit for bit."""
import numpy as np
import pytest
import torch

import midas_ref
import synth
import vslam_abi

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _s():
    """torch's current stream: the library's launches are ordered after the tensors' uploads."""
    return torch.cuda.current_stream().cuda_stream


@pytest.fixture(scope="module")
def midas(vsctx):
    m = vslam_abi.Midas(vsctx)
    yield m
    m.close()


@pytest.fixture(scope="module")
def hd_frames():
    L = synth.loop_sequence(3, workers=3, K=synth.K_HD, w=synth.W_HD, h=synth.H_HD)
    return L["bgr"]


def _pre_dev(midas, bgr):
    B, h, w = bgr.shape[:3]
    d_bgr = torch.from_numpy(np.ascontiguousarray(bgr)).to(DEV)
    out = torch.zeros((B, 256, 256, 3), dtype=torch.float32, device=DEV)
    midas.preprocess_dev(B, d_bgr.data_ptr(), h, w, out.data_ptr(), _s())
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("shape", [(720, 1280), (480, 640), (97, 131)])
def test_preprocess_bit_exact(midas, shape):
    h, w = shape
    rng = np.random.default_rng(h)
    bgr = rng.integers(0, 256, (2, h, w, 3), dtype=np.uint8)
    got = _pre_dev(midas, bgr)
    for b in range(2):
        assert np.array_equal(got[b].view(np.uint32), midas_ref.preprocess(bgr[b]).view(np.uint32))


def test_network_matches_torch_fp64(midas, hd_frames):
    x = midas_ref.preprocess(hd_frames[0])[None]  # [1, 256, 256, 3]
    d_in = torch.from_numpy(x).to(DEV).contiguous()
    d_out = torch.zeros((1, 256, 256), dtype=torch.float32, device=DEV)
    midas.forward_dev(1, d_in.data_ptr(), d_out.data_ptr(), _s())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()[0]
    ref = midas_ref.forward(midas.weights(), torch.from_numpy(x).permute(0, 3, 1, 2)).numpy()[0]
    rng_ = float(ref.max() - ref.min())
    err = float(np.abs(got - ref).max())
    print(f"MiDaS network: max |gpu - fp64| = {err:.3e}, output range {rng_:.3e}")
    assert rng_ > 0
    assert err <= 1e-4 * rng_


def test_postprocess_matches_restatement(midas):
    rng = np.random.default_rng(5)
    small = rng.random((2, 256, 256), dtype=np.float32) * 3.0
    for h, w in [(720, 1280), (480, 640)]:
        d_s = torch.from_numpy(small).to(DEV)
        d_o = torch.zeros((2, h, w), dtype=torch.float32, device=DEV)
        midas.postprocess_dev(2, d_s.data_ptr(), h, w, d_o.data_ptr(), _s())
        torch.cuda.synchronize()
        got = d_o.cpu().numpy()
        for b in range(2):
            ref = midas_ref.postprocess(small[b], h, w)
            assert np.abs(got[b] - ref).max() <= 2e-6
            # fma(d, (float)(1/range), (float)(-min/range)): the ends are 0 and 1 up to that rounding
            assert abs(float(got[b].min())) <= 1e-6 and abs(float(got[b].max()) - 1.0) <= 1e-6


def test_estimate_is_the_chained_stages_and_batch_independent(midas, hd_frames):
    h, w = hd_frames.shape[1:3]
    d_bgr = torch.from_numpy(np.ascontiguousarray(hd_frames)).to(DEV)
    B = d_bgr.shape[0]
    full = torch.zeros((B, h, w), dtype=torch.float32, device=DEV)
    midas.estimate_dev(B, d_bgr.data_ptr(), h, w, full.data_ptr(), _s())
    one = torch.zeros((1, h, w), dtype=torch.float32, device=DEV)
    x = torch.zeros((1, 256, 256, 3), dtype=torch.float32, device=DEV)
    small = torch.zeros((1, 256, 256), dtype=torch.float32, device=DEV)
    staged = torch.zeros((1, h, w), dtype=torch.float32, device=DEV)
    for b in range(B):
        midas.estimate_dev(1, d_bgr[b].data_ptr(), h, w, one.data_ptr(), _s())
        midas.preprocess_dev(1, d_bgr[b].data_ptr(), h, w, x.data_ptr(), _s())
        midas.forward_dev(1, x.data_ptr(), small.data_ptr(), _s())
        midas.postprocess_dev(1, small.data_ptr(), h, w, staged.data_ptr(), _s())
        torch.cuda.synchronize()
        assert torch.equal(one[0], full[b]) and torch.equal(staged[0], full[b])
    f = full.cpu().numpy()
    assert f.min() >= -1e-6 and f.max() <= 1.0 + 1e-6


def test_weight_file_round_trip(vsctx, midas, hd_frames, tmp_path):
    p = tmp_path / "m.vsmw"
    midas.save_weights(p)
    h, w = hd_frames.shape[1:3]
    d_bgr = torch.from_numpy(np.ascontiguousarray(hd_frames[:1])).to(DEV)
    a = torch.zeros((1, h, w), dtype=torch.float32, device=DEV)
    b = torch.zeros_like(a)
    midas.estimate_dev(1, d_bgr.data_ptr(), h, w, a.data_ptr(), _s())
    with vslam_abi.Midas(vsctx, str(p)) as m2:
        m2.estimate_dev(1, d_bgr.data_ptr(), h, w, b.data_ptr(), _s())
        torch.cuda.synchronize()
    assert torch.equal(a, b)
    bad = tmp_path / "bad.vsmw"
    bad.write_bytes(b"VSMWxxxx")
    with pytest.raises(vslam_abi.VSError, match="VS_ERR_IO"):
        vslam_abi.Midas(vsctx, str(bad))
