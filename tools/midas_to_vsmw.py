"""Convert a MiDaS v2.1-small state_dict (midas_v21_small_256.pt: MidasNet_small, EfficientNet-Lite3
backbone from timm tf_efficientnet_lite3) into the library's VSMW weight file: BatchNorm (eps 1e-3,
the TF-ported timm default) folded into the preceding convolution, layers in the order of
csrc/midas.hip's builder (tests/midas_ref.py restates it), conv weights [cout][cin][k][k] + bias,
depthwise [c][k][k] + bias.  scratch.refinenet4.resConfUnit1 is not used by the forward pass
(refinenet4 has one input) and is skipped, as the reference's ONNX export drops it.

The checkpoint is read with torch.load(weights_only=True) (no code executed from the file).

    python tools/midas_to_vsmw.py midas_v21_small_256.pt out.vsmw
"""
import sys

import numpy as np

BN_EPS = 1e-3
# (state_dict group, channels) of the six InvertedResidual stages after the DepthwiseSeparable one
STAGE_GROUPS = ["pretrained.layer1.4", "pretrained.layer2.0", "pretrained.layer3.0", "pretrained.layer3.1",
                "pretrained.layer4.0", "pretrained.layer4.1"]
STAGE_REPEATS = [3, 3, 5, 5, 6, 1]


def _np(t):
    return t.detach().cpu().double().numpy() if hasattr(t, "detach") else np.asarray(t, np.float64)


def convert(sd):
    """state_dict (name -> tensor) -> flat float32 canonical weights."""
    out = []
    used = set()

    def get(k):
        if k not in sd:
            raise KeyError(f"missing {k}")
        used.add(k)
        return _np(sd[k])

    def fold(w, bn):
        g, b, m, v = get(bn + ".weight"), get(bn + ".bias"), get(bn + ".running_mean"), get(bn + ".running_var")
        s = g / np.sqrt(v + BN_EPS)
        return w * s.reshape(-1, *([1] * (w.ndim - 1))), b - m * s

    def conv_bn(wk, bn):
        w, b = fold(get(wk), bn)
        out.extend([w.ravel(), b])

    def dw_bn(wk, bn):
        w, b = fold(get(wk), bn)  # [c, 1, k, k]
        out.extend([w.ravel(), b])

    def conv(prefix, bias=True):
        out.append(get(prefix + ".weight").ravel())
        if bias:
            out.append(get(prefix + ".bias"))

    conv_bn("pretrained.layer1.0.weight", "pretrained.layer1.1")  # conv_stem + bn1
    ds = "pretrained.layer1.3.0"
    dw_bn(ds + ".conv_dw.weight", ds + ".bn1")
    conv_bn(ds + ".conv_pw.weight", ds + ".bn2")
    for g, n in zip(STAGE_GROUPS, STAGE_REPEATS):
        for i in range(n):
            p = f"{g}.{i}"
            conv_bn(p + ".conv_pw.weight", p + ".bn1")
            dw_bn(p + ".conv_dw.weight", p + ".bn2")
            conv_bn(p + ".conv_pwl.weight", p + ".bn3")
    for i in range(1, 5):
        conv(f"scratch.layer{i}_rn", bias=False)

    def rcu(p):
        conv(p + ".conv1")
        conv(p + ".conv2")

    rcu("scratch.refinenet4.resConfUnit2")
    conv("scratch.refinenet4.out_conv")
    for r in (3, 2, 1):
        rcu(f"scratch.refinenet{r}.resConfUnit1")
        rcu(f"scratch.refinenet{r}.resConfUnit2")
        conv(f"scratch.refinenet{r}.out_conv")
    for i in (0, 2, 4):
        conv(f"scratch.output_conv.{i}")
    skipped = [k for k in sd if k not in used and not k.endswith("num_batches_tracked")
               and not k.startswith("scratch.refinenet4.resConfUnit1.")]
    if skipped:
        raise KeyError(f"unexpected keys (not MiDaS v2.1 small?): {skipped[:8]}")
    return np.concatenate(out).astype(np.float32)


def write_vsmw(path, flat):
    with open(path, "wb") as f:
        f.write(np.array([0x574D5356, 1], "<u4").tobytes() + np.array([flat.size], "<u8").tobytes())
        f.write(flat.astype("<f4").tobytes())


def main():
    import torch
    src, dst = sys.argv[1], sys.argv[2]
    sd = torch.load(src, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    flat = convert(sd)
    write_vsmw(dst, flat)
    print(f"{dst}: {flat.size} parameters")


if __name__ == "__main__":
    main()
