"""MiDaS v2.1-small (F3, reference src/DepthEstimator.cpp:39-112) — CPU checks:

* the torch restatement (tests/midas_ref.py) and the library's builder (csrc/midas.hip) agree on
  the parameter count of the topology;
* tools/midas_to_vsmw.py: a synthetic state_dict with MiDaS v2.1-small's key layout (timm
  tf_efficientnet_lite3 block names, scratch.* decoder names, random BatchNorm statistics) run
  through an unfused forward (conv + BatchNorm(eps 1e-3), written here from the state_dict keys)
  equals tests/midas_ref.py on the converted, BatchNorm-folded weights;
* the pre-processing restatement keeps the reference's quirks (BGR planes normalised with the
  RGB-ordered ImageNet constants, :54-58) and its shape.
No real checkpoint is available offline (README.md:43: weights not shipped), so the key layout is
the published one, not one read from a file ("parity unpinned" for real weights)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import midas_ref

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_param_count_matches_library():
    import vslam_abi
    assert midas_ref.num_params() == vslam_abi.Midas.num_params() == 16563873


def _fake_state_dict(seed=0):
    g = torch.Generator().manual_seed(seed)
    sd = {}

    def conv(name, cout, cin, k, bias=True, groups=1):
        sd[name + ".weight"] = torch.randn(cout, cin // groups, k, k, generator=g) * (2.0 / (cin // groups * k * k)) ** 0.5
        if bias:
            sd[name + ".bias"] = torch.randn(cout, generator=g) * 0.05

    def bn(name, c):
        sd[name + ".weight"] = 1.0 + 0.1 * torch.randn(c, generator=g)
        sd[name + ".bias"] = 0.1 * torch.randn(c, generator=g)
        sd[name + ".running_mean"] = 0.1 * torch.randn(c, generator=g)
        sd[name + ".running_var"] = 0.5 + torch.rand(c, generator=g)
        sd[name + ".num_batches_tracked"] = torch.tensor(0)

    conv("pretrained.layer1.0", 32, 3, 3, bias=False)
    bn("pretrained.layer1.1", 32)
    conv("pretrained.layer1.3.0.conv_dw", 32, 32, 3, bias=False, groups=32)
    bn("pretrained.layer1.3.0.bn1", 32)
    conv("pretrained.layer1.3.0.conv_pw", 24, 32, 1, bias=False)
    bn("pretrained.layer1.3.0.bn2", 24)
    from midas_to_vsmw import STAGE_GROUPS, STAGE_REPEATS
    cin = 24
    for grp, n, (c, k, s, _) in zip(STAGE_GROUPS, STAGE_REPEATS, midas_ref.STAGES):
        for i in range(n):
            p = f"{grp}.{i}"
            e = cin * 6
            conv(p + ".conv_pw", e, cin, 1, bias=False)
            bn(p + ".bn1", e)
            conv(p + ".conv_dw", e, e, k, bias=False, groups=e)
            bn(p + ".bn2", e)
            conv(p + ".conv_pwl", c, e, 1, bias=False)
            bn(p + ".bn3", c)
            cin = c
    for i, (ci, co) in enumerate(((32, 64), (48, 128), (136, 256), (384, 512)), 1):
        conv(f"scratch.layer{i}_rn", co, ci, 3, bias=False)
    for r, c, out in ((4, 512, 256), (3, 256, 128), (2, 128, 64), (1, 64, 64)):
        for u in (1, 2):  # refinenet4.resConfUnit1 exists in the checkpoint but is unused
            conv(f"scratch.refinenet{r}.resConfUnit{u}.conv1", c, c, 3)
            conv(f"scratch.refinenet{r}.resConfUnit{u}.conv2", c, c, 3)
        conv(f"scratch.refinenet{r}.out_conv", out, c, 1)
    conv("scratch.output_conv.0", 32, 64, 3)
    conv("scratch.output_conv.2", 32, 32, 3)
    conv("scratch.output_conv.4", 1, 32, 1)
    return sd


def _forward_state_dict(sd, x):
    """MidasNet_small.forward straight from the state_dict (unfused BatchNorm), float64."""
    P = {k: v.double() for k, v in sd.items()}

    def bn(y, n):
        return F.batch_norm(y, P[n + ".running_mean"], P[n + ".running_var"], P[n + ".weight"], P[n + ".bias"],
                            False, 0.0, 1e-3)

    def same_conv(y, w, stride, groups=1):
        k = w.shape[-1]
        pt, pb = midas_ref._same(y.shape[2], k, stride)
        pl, pr = midas_ref._same(y.shape[3], k, stride)
        return F.conv2d(F.pad(y, (pl, pr, pt, pb)), w, None, stride=stride, groups=groups)

    def conv(y, n, relu_in=False):
        if relu_in:
            y = F.relu(y)
        w = P[n + ".weight"]
        return F.conv2d(y, w, P.get(n + ".bias"), padding=w.shape[-1] // 2)

    y = F.relu6(bn(same_conv(x, P["pretrained.layer1.0.weight"], 2), "pretrained.layer1.1"))
    d = "pretrained.layer1.3.0"
    y = F.relu6(bn(same_conv(y, P[d + ".conv_dw.weight"], 1, groups=y.shape[1]), d + ".bn1"))
    y = bn(F.conv2d(y, P[d + ".conv_pw.weight"]), d + ".bn2")
    from midas_to_vsmw import STAGE_GROUPS, STAGE_REPEATS
    skips = []
    for si, (grp, n, (c, k, s, _)) in enumerate(zip(STAGE_GROUPS, STAGE_REPEATS, midas_ref.STAGES)):
        for i in range(n):
            p = f"{grp}.{i}"
            stride = s if i == 0 else 1
            h = F.relu6(bn(F.conv2d(y, P[p + ".conv_pw.weight"]), p + ".bn1"))
            h = F.relu6(bn(same_conv(h, P[p + ".conv_dw.weight"], stride, groups=h.shape[1]), p + ".bn2"))
            h = bn(F.conv2d(h, P[p + ".conv_pwl.weight"]), p + ".bn3")
            y = h + y if (stride == 1 and y.shape[1] == c) else h
        if si in (0, 1, 3, 5):
            skips.append(y)
    rn = [conv(t, f"scratch.layer{i}_rn") for i, t in enumerate(skips, 1)]

    def rcu(t, n):
        return conv(F.relu(conv(t, n + ".conv1", relu_in=True)), n + ".conv2") + t

    def fusion(r, xs0, xs1):
        o = xs0
        if xs1 is not None:
            o = o + rcu(xs1, f"scratch.refinenet{r}.resConfUnit1")
        o = rcu(o, f"scratch.refinenet{r}.resConfUnit2")
        o = F.interpolate(o, scale_factor=2, mode="bilinear", align_corners=True)
        return conv(o, f"scratch.refinenet{r}.out_conv")

    p4 = fusion(4, rn[3], None)
    p3 = fusion(3, p4, rn[2])
    p2 = fusion(2, p3, rn[1])
    p1 = fusion(1, p2, rn[0])
    o = conv(p1, "scratch.output_conv.0")
    o = F.interpolate(o, scale_factor=2, mode="bilinear", align_corners=False)
    o = F.relu(conv(o, "scratch.output_conv.2"))
    o = F.relu(conv(o, "scratch.output_conv.4"))
    return o[:, 0]


def test_converter_folds_batchnorm_into_the_canonical_layout():
    from midas_to_vsmw import convert
    sd = _fake_state_dict()
    flat = convert(sd)
    assert flat.size == midas_ref.num_params()
    x = torch.randn(1, 3, 64, 64, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    ref = _forward_state_dict(sd, x)
    got = midas_ref.forward(flat, x)
    scale = float(ref.abs().max())
    assert scale > 0
    assert float((got - ref).abs().max()) <= 1e-5 * scale


def test_converter_rejects_foreign_keys():
    from midas_to_vsmw import convert
    sd = _fake_state_dict()
    sd["scratch.something_else.weight"] = torch.zeros(1)
    with pytest.raises(KeyError):
        convert(sd)
    sd = _fake_state_dict()
    del sd["scratch.output_conv.4.bias"]
    with pytest.raises(KeyError):
        convert(sd)


def test_preprocess_restatement_shape_and_channel_order():
    rng = np.random.default_rng(0)
    bgr = rng.integers(0, 256, (720, 1280, 3), dtype=np.uint8)
    x = midas_ref.preprocess(bgr)
    assert x.shape == (256, 256, 3) and x.dtype == np.float32
    flat = np.zeros((720, 1280, 3), np.uint8)
    flat[..., 0] = 255  # pure blue in BGR: plane 0 normalised with the R constants (0.485, 0.229)
    v = midas_ref.preprocess(flat)
    assert np.allclose(v[..., 0], (1 - 0.485) / 0.229, atol=1e-5)
    assert np.allclose(v[..., 2], (0 - 0.406) / 0.225, atol=1e-5)
