"""vs_create / vs_midas_create on the reference's own kind of model file (VERDICT r02 missing #1):
an ONNX SuperPoint / MiDaS export (hand-encoded by tests/onnx_writer.py from the library's seeded
weights) must give bit-identical keypoints, descriptors and depth to the seeded-weight path.
Reference: Slam.cpp:28-31, FeatureExtractor.cpp:22-44, DepthEstimator.cpp:15-36."""
import numpy as np
import pytest

import onnx_writer
import vslam_abi

pytestmark = pytest.mark.gpu


def test_vs_create_loads_superpoint_onnx(tmp_path, vsctx, seq4):
    p = tmp_path / "superpoint_v1.onnx"
    p.write_bytes(onnx_writer.superpoint_model(vslam_abi.superpoint_synth_weights(), heads_swapped=True))
    with vslam_abi.Context(0, str(p)) as c:
        assert np.array_equal(c.weights().view(np.uint32), vsctx.weights().view(np.uint32))
        imgs = [f["bgr"] for f in seq4]
        for (ka, da), (kb, db) in zip(c.extract_batch(imgs), vsctx.extract_batch(imgs)):
            assert len(ka) == len(kb) > 0
            assert np.array_equal(ka.view(np.uint8), kb.view(np.uint8))
            assert np.array_equal(da.view(np.uint32), db.view(np.uint32))


def test_vs_create_reports_a_bad_onnx(tmp_path):
    p = tmp_path / "broken.onnx"
    p.write_bytes(onnx_writer.superpoint_model(vslam_abi.superpoint_synth_weights(), drop_pool=True))
    with pytest.raises(vslam_abi.VSError, match="IO"):
        vslam_abi.Context(0, str(p))


def test_vs_midas_create_loads_midas_onnx(tmp_path, vsctx):
    import torch
    import synth
    p = tmp_path / "midas_v21_small_256.onnx"
    p.write_bytes(onnx_writer.midas_model(vslam_abi.midas_synth_weights(), bn_every=2))
    L = synth.loop_sequence(2, workers=2)
    dev = torch.device("cuda", 0)
    bgr = torch.from_numpy(L["bgr"]).to(dev)
    outs = []
    for path in (str(p), None):
        with vslam_abi.Midas(vsctx, path) as m:
            d = torch.zeros((2, 480, 640), dtype=torch.float32, device=dev)
            m.estimate_dev(2, bgr.data_ptr(), 480, 640, d.data_ptr())
            torch.cuda.synchronize()
            outs.append((m.weights(), d.cpu().numpy()))
    assert np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32))
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))
    assert np.ptp(outs[0][1]) > 0
