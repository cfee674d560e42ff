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


# ---- output tails: the reference samples whatever "desc" the graph returns -----
@pytest.mark.parametrize("tail", [t for t in onnx_writer.DESC_TAILS])
def test_superpoint_onnx_desc_tail_is_classified(tmp_path, sp_weights, tail):
    p = tmp_path / f"sp_{tail}.onnx"
    p.write_bytes(onnx_writer.superpoint_model(sp_weights, desc_tail=tail, seed=2))
    assert vslam_abi.superpoint_onnx_desc_normalized(str(p)) == (tail != "raw")
    got = vslam_abi.superpoint_onnx_weights(str(p))
    assert np.array_equal(got.view(np.uint32), sp_weights.view(np.uint32))


@pytest.mark.parametrize("kw,msg", [(dict(semi_tail="softmax"), "raw logits"),
                                    (dict(desc_tail="reduce_all"), "L2 normalisation over channels"),
                                    (dict(desc_tail="pow3_sum_sqrt"), "L2 normalisation over channels"),
                                    (dict(desc_tail="pow_int3_sum_sqrt"), "L2 normalisation over channels"),
                                    (dict(desc_tail="clip_max"), "L2 normalisation over channels"),
                                    (dict(pads=False), "explicit pads")])
def test_superpoint_onnx_rejects_other_tails_and_default_padding(tmp_path, sp_weights, kw, msg):
    p = tmp_path / "bad.onnx"
    p.write_bytes(onnx_writer.superpoint_model(sp_weights, **kw))
    with pytest.raises(vslam_abi.VSError, match=msg):
        vslam_abi.superpoint_onnx_weights(str(p))
    with pytest.raises(vslam_abi.VSError, match="IO"):
        vslam_abi.superpoint_onnx_desc_normalized(str(p))


def test_midas_onnx_rejects_rewired_and_unpadded_graphs(tmp_path, midas_w):
    p = tmp_path / "midas_swapped.onnx"
    p.write_bytes(onnx_writer.midas_model(midas_w, swap_fusion3=True))
    with pytest.raises(vslam_abi.VSError, match="wired"):
        vslam_abi.midas_onnx_weights(str(p))
    q = tmp_path / "midas_nopad.onnx"
    q.write_bytes(onnx_writer.midas_model(midas_w, drop_stem_pad=True))
    with pytest.raises(vslam_abi.VSError, match="Pad"):
        vslam_abi.midas_onnx_weights(str(q))


# ---- hostile files: errors, never a crash or an exception through the C ABI ------
def _model_with_tensor(dims, payload=b"", dtype=1, extra_nodes=()):
    w = onnx_writer
    t = w._ld(1, b"".join(w._varint(d) for d in dims)) + w._i(2, dtype) + w._s(8, "W") + w._ld(9, payload)
    conv = w.node("Conv", ["image", "W"], ["semi"], attrs=[w.attr_ints("kernel_shape", [3, 3])])
    return w.model([conv] + list(extra_nodes), [t], ["image"], ["semi"])


@pytest.mark.parametrize("dims", [[1 << 40, 1 << 30], [-5, 3], [1 << 62, 4, 4, 4], [64, 1, 3, 3]])
def test_onnx_reader_survives_hostile_tensor_dims(tmp_path, dims):
    p = tmp_path / "hostile.onnx"
    p.write_bytes(_model_with_tensor(dims, payload=b"\0" * 16))
    with pytest.raises(vslam_abi.VSError, match="IO"):
        vslam_abi.superpoint_onnx_weights(str(p))


def test_onnx_reader_survives_input_less_nodes(tmp_path):
    w = onnx_writer
    # a Conv whose weight comes from an input-less Identity, and a Relu with no inputs feeding it
    nodes = [w.node("Identity", [], ["Wi"]), w.node("Relu", [], ["x"]),
             w.node("Conv", ["x", "Wi"], ["semi"], attrs=[w.attr_ints("kernel_shape", [3, 3])])]
    p = tmp_path / "inputless.onnx"
    p.write_bytes(w.model(nodes, [], ["image"], ["semi"]))
    with pytest.raises(vslam_abi.VSError, match="IO"):
        vslam_abi.superpoint_onnx_weights(str(p))
    with pytest.raises(vslam_abi.VSError, match="IO"):
        vslam_abi.midas_onnx_weights(str(p))


def test_onnx_reader_rejects_auto_pad(tmp_path):
    w = onnx_writer
    # an auto_pad=SAME_UPPER Conv appended to an otherwise valid graph
    t = w.tensor("Wx", np.zeros((1, 1, 3, 3), np.float32))
    conv = w.node("Conv", ["image", "Wx"], ["extra"], attrs=[w.attr_ints("kernel_shape", [3, 3]),
                                                              w._s(1, "auto_pad") + w._i(20, 3) + w._s(4, "SAME_UPPER")])
    p = tmp_path / "autopad.onnx"
    p.write_bytes(w.model([conv], [t], ["image"], ["extra"]))
    with pytest.raises(vslam_abi.VSError, match="auto_pad"):
        vslam_abi.superpoint_onnx_weights(str(p))
