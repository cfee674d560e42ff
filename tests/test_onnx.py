"""The library's ONNX reader (host/onnx_weights.cpp) on hand-encoded model files
(tests/onnx_writer.py; the `onnx` package is absent): the weights vs_create / vs_midas_create take
from the reference's own model files (models/superpoint_v1.onnx, models/midas_v21_small_256.onnx;
Slam.cpp:28-31, FeatureExtractor.cpp:22-44, DepthEstimator.cpp:15-36).  Host only — no GPU."""
import numpy as np
import pytest

import onnx_writer
import vslam_abi


@pytest.fixture(scope="module")
def sp_weights():
    return vslam_abi.superpoint_synth_weights()


@pytest.fixture(scope="module")
def midas_w():
    return vslam_abi.midas_synth_weights()


@pytest.mark.parametrize("variant", [dict(), dict(heads_swapped=True, seed=3), dict(modes=["unpacked"], seed=5),
                                     dict(modes=["packed", "raw"], identity_alias=False, seed=9)])
def test_superpoint_onnx_round_trip(tmp_path, sp_weights, variant):
    p = tmp_path / "superpoint_v1.onnx"
    p.write_bytes(onnx_writer.superpoint_model(sp_weights, **variant))
    got = vslam_abi.superpoint_onnx_weights(str(p))
    assert np.array_equal(got.view(np.uint32), sp_weights.view(np.uint32))


def test_superpoint_onnx_float16_weights(tmp_path, sp_weights):
    p = tmp_path / "sp16.onnx"
    p.write_bytes(onnx_writer.superpoint_model(sp_weights, modes=["f16"]))
    got = vslam_abi.superpoint_onnx_weights(str(p))
    assert np.array_equal(got, sp_weights.astype(np.float16).astype(np.float32))


def test_superpoint_onnx_mapping_is_structural(tmp_path):
    """Weights are placed by graph structure, not by initializer names or order: distinct values
    per layer land in their canonical slots whatever the head order."""
    n = vslam_abi.load_library().vs_superpoint_num_params()
    flat, o = np.zeros(n, np.float32), 0
    for li, (cin, cout, k) in enumerate(onnx_writer.SP_LAYERS):
        m = cout * cin * k * k + cout
        flat[o:o + m] = li + np.arange(m, dtype=np.float32) * 1e-6
        o += m
    for swapped in (False, True):
        p = tmp_path / f"s{swapped}.onnx"
        p.write_bytes(onnx_writer.superpoint_model(flat, heads_swapped=swapped, seed=11))
        assert np.array_equal(vslam_abi.superpoint_onnx_weights(str(p)), flat)


def test_superpoint_onnx_rejects_other_graphs(tmp_path, sp_weights):
    bad = tmp_path / "nopool.onnx"
    bad.write_bytes(onnx_writer.superpoint_model(sp_weights, drop_pool=True))
    with pytest.raises(vslam_abi.VSError, match="backbone"):
        vslam_abi.superpoint_onnx_weights(str(bad))
    trunc = tmp_path / "trunc.onnx"
    trunc.write_bytes(onnx_writer.superpoint_model(sp_weights)[:100000])
    with pytest.raises(vslam_abi.VSError):
        vslam_abi.superpoint_onnx_weights(str(trunc))
    with pytest.raises(vslam_abi.VSError, match="cannot open"):
        vslam_abi.superpoint_onnx_weights(str(tmp_path / "missing.onnx"))
    mid = tmp_path / "midas_as_sp.onnx"
    mid.write_bytes(onnx_writer.midas_model(vslam_abi.midas_synth_weights()))
    with pytest.raises(vslam_abi.VSError, match="12 convolutions"):
        vslam_abi.superpoint_onnx_weights(str(mid))


def test_midas_onnx_round_trip_with_batchnorm(tmp_path, midas_w):
    for bn_every in (0, 2, 1):
        p = tmp_path / f"midas_{bn_every}.onnx"
        p.write_bytes(onnx_writer.midas_model(midas_w, bn_every=bn_every, seed=bn_every))
        got = vslam_abi.midas_onnx_weights(str(p))
        assert np.array_equal(got.view(np.uint32), midas_w.view(np.uint32)), bn_every


def test_midas_onnx_folds_batchnorm_statistics(tmp_path, midas_w):
    """Random BatchNormalization statistics (epsilon 1e-3): the reader folds them as
    w * g / sqrt(var + eps), beta - mean * g / sqrt(var + eps) in double, like
    tools/midas_to_vsmw.py."""
    rec = {}
    p = tmp_path / "midas_bn.onnx"
    p.write_bytes(onnx_writer.midas_model(midas_w, bn_every=3, seed=4, bn_random=rec))
    got = vslam_abi.midas_onnx_weights(str(p))
    want = midas_w.copy()
    for off, wf, bf in rec["folded"]:
        want[off:off + wf.size] = wf.reshape(-1)
        want[off + wf.size:off + wf.size + bf.size] = bf
    assert len(rec["folded"]) > 20
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_midas_onnx_rejects_wrong_network(tmp_path, sp_weights):
    p = tmp_path / "sp_as_midas.onnx"
    p.write_bytes(onnx_writer.superpoint_model(sp_weights))
    with pytest.raises(vslam_abi.VSError, match="MiDaS graph"):
        vslam_abi.midas_onnx_weights(str(p))
