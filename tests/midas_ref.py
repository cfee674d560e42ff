"""Torch (CPU, float64 by default) restatement of the MiDaS v2.1-small network the library runs
(csrc/midas.hip; published topology: MidasNet_small(features=64, backbone="efficientnet_lite3",
expand=True, non_negative=True) over timm's tf_efficientnet_lite3), reading the library's
canonical flat weights (BatchNorm folded), plus numpy restatements of the reference's pre- and
post-processing (src/DepthEstimator.cpp:39-112).  Test infrastructure only.

The topology here is written independently of the C++ builder; tests/test_midas.py checks that
both agree on the parameter count, and the GPU tests compare activations."""
import math

import numpy as np
import torch
import torch.nn.functional as F

STAGES = [(32, 3, 2, 3), (48, 5, 2, 3), (96, 3, 2, 5), (136, 5, 1, 5), (232, 5, 2, 6), (384, 3, 1, 1)]


def _same(i, k, s):
    o = (i + s - 1) // s
    total = max((o - 1) * s + k - i, 0)
    return total // 2, total - total // 2


class _W:
    def __init__(self, flat, dtype):
        self.flat = torch.as_tensor(np.asarray(flat, np.float32)).to(dtype)
        self.p = 0

    def take(self, n, shape):
        t = self.flat[self.p:self.p + n].reshape(shape)
        self.p += n
        return t


def forward(weights, x, dtype=torch.float64, trace=None):
    """weights: flat canonical array; x: [B, 3, 256, 256] (NCHW, normalised).  Returns [B, 256, 256].
    trace: a list that receives every step's output (conv / depthwise / upsample, library order)."""
    W = _W(weights, dtype)
    x = torch.as_tensor(x).to(dtype)

    def rec(y):
        if trace is not None:
            trace.append(y)
        return y

    def conv(x, cout, k, stride=1, act=None, tf_same=False, bias=True, res1=None, res2=None, pre_relu=False):
        cin = x.shape[1]
        w = W.take(cout * cin * k * k, (cout, cin, k, k))
        b = W.take(cout, (cout,)) if bias else None
        if pre_relu:
            x = F.relu(x)
        if tf_same:
            pt, pb = _same(x.shape[2], k, stride)
            pl, pr = _same(x.shape[3], k, stride)
            y = F.conv2d(F.pad(x, (pl, pr, pt, pb)), w, b, stride=stride)
        else:
            y = F.conv2d(x, w, b, stride=stride, padding=k // 2)
        if act == "relu":
            y = F.relu(y)
        elif act == "relu6":
            y = F.relu6(y)
        if res1 is not None:
            y = y + res1
        if res2 is not None:
            y = res2 + y
        return rec(y)

    def dw(x, k, stride):
        c = x.shape[1]
        w = W.take(c * k * k, (c, 1, k, k))
        b = W.take(c, (c,))
        pt, pb = _same(x.shape[2], k, stride)
        pl, pr = _same(x.shape[3], k, stride)
        return rec(F.relu6(F.conv2d(F.pad(x, (pl, pr, pt, pb)), w, b, stride=stride, groups=c)))

    def ir(x, cout, k, stride):
        cin = x.shape[1]
        h = conv(x, cin * 6, 1, act="relu6")
        h = dw(h, k, stride)
        return conv(h, cout, 1, res1=x if (stride == 1 and cin == cout) else None)

    def rcu(x, extra=None):
        c = x.shape[1]
        h = conv(x, c, 3, act="relu", pre_relu=True)
        return conv(h, c, 3, res1=x, res2=extra)

    def fusion(xs0, xs1, out_ch):
        o = rcu(xs1, xs0) if xs1 is not None else xs0
        o = rcu(o)
        o = rec(F.interpolate(o, scale_factor=2, mode="bilinear", align_corners=True))
        return conv(o, out_ch, 1)

    h = conv(x, 32, 3, 2, act="relu6", tf_same=True)
    h = dw(h, 3, 1)
    h = conv(h, 24, 1)
    skips = []
    for si, (c, k, s, n) in enumerate(STAGES):
        for r in range(n):
            h = ir(h, c, k, s if r == 0 else 1)
        if si in (0, 1, 3, 5):
            skips.append(h)
    rn = [conv(t, c, 3, bias=False) for t, c in zip(skips, (64, 128, 256, 512))]
    p4 = fusion(rn[3], None, 256)
    p3 = fusion(p4, rn[2], 128)
    p2 = fusion(p3, rn[1], 64)
    p1 = fusion(p2, rn[0], 64)
    o = conv(p1, 32, 3)
    o = rec(F.interpolate(o, scale_factor=2, mode="bilinear", align_corners=False))
    o = conv(o, 32, 3, act="relu")
    o = conv(o, 1, 1, act="relu")
    assert W.p == W.flat.numel(), (W.p, W.flat.numel())
    return o[:, 0]


def num_params():
    n = 0

    def conv(cin, cout, k, bias=True):
        return cout * cin * k * k + (cout if bias else 0)

    n += conv(3, 32, 3) + 32 * 9 + 32 + conv(32, 24, 1)
    cin = 24
    for c, k, s, reps in STAGES:
        for r in range(reps):
            e = cin * 6
            n += conv(cin, e, 1) + e * k * k + e + conv(e, c, 1)
            cin = c
    for ci, co in ((32, 64), (48, 128), (136, 256), (384, 512)):
        n += conv(ci, co, 3, bias=False)
    for c, out, rcus in ((512, 256, 1), (256, 128, 2), (128, 64, 2), (64, 64, 2)):
        n += rcus * 2 * conv(c, c, 3) + conv(c, out, 1)
    n += conv(64, 32, 3) + conv(32, 32, 3) + conv(32, 1, 1)
    return n


# ---- pre / post-processing (DepthEstimator.cpp:49-67, 96-109) ----------------------------------
def _lin(n_dst, n_src):
    """OpenCV resizeGeneric_ INTER_LINEAR coefficients: (s0, s1, f float32)."""
    scale = 1.0 / (n_dst / n_src)
    d = np.arange(n_dst)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0.0, 0
    hi = s >= n_src - 1
    f[hi], s[hi] = 0.0, n_src - 1
    return s, np.minimum(s + 1, n_src - 1), f


def preprocess(bgr):
    """[h, w, 3] u8 -> [256, 256, 3] float32: 8-bit INTER_LINEAR resize (VResizeLinearVec_32s8u row
    formula), *(float)(1/255), fma with (float)(1/std), (float)(-mean/std) per BGR plane."""
    h, w = bgr.shape[:2]
    sx0, sx1, fx = _lin(256, w)
    sy0, sy1, fy = _lin(256, h)
    a0 = np.rint(((np.float32(1) - fx) * np.float32(2048))).astype(np.int64)
    a1 = np.rint((fx * np.float32(2048))).astype(np.int64)
    b0 = np.rint(((np.float32(1) - fy) * np.float32(2048))).astype(np.int64)
    b1 = np.rint((fy * np.float32(2048))).astype(np.int64)
    img = bgr.astype(np.int64)
    hr0 = img[sy0][:, sx0] * a0[None, :, None] + img[sy0][:, sx1] * a1[None, :, None]
    hr1 = img[sy1][:, sx0] * a0[None, :, None] + img[sy1][:, sx1] * a1[None, :, None]
    v = (((hr0 >> 4) * b0[:, None, None]) >> 16) + (((hr1 >> 4) * b1[:, None, None]) >> 16)
    v = np.clip((v + 2) >> 2, 0, 255).astype(np.float32)
    f = (v * np.float32(1.0 / 255.0)).astype(np.float32)
    mean = np.array([0.485, 0.456, 0.406], np.float32).astype(np.float64)
    std = np.array([0.229, 0.224, 0.225], np.float32).astype(np.float64)
    inv = 1.0 / std
    A = inv.astype(np.float32).astype(np.float64)
    Bc = (-mean * inv).astype(np.float32).astype(np.float64)
    return np.ascontiguousarray((f.astype(np.float64) * A + Bc).astype(np.float32))  # fma: one rounding


def postprocess(small, h, w):
    """[256, 256] float32 -> [h, w] float32 in [0, 1] (float INTER_LINEAR resize, min-max)."""
    sx0, sx1, fx = _lin(w, 256)
    sy0, sy1, fy = _lin(h, 256)
    s = small.astype(np.float32)
    a0, a1 = np.float32(1) - fx, fx
    b0, b1 = np.float32(1) - fy, fy
    r0 = s[sy0][:, sx0] * a0 + s[sy0][:, sx1] * a1
    r1 = s[sy1][:, sx0] * a0 + s[sy1][:, sx1] * a1
    d = (r0 * b0[:, None] + r1 * b1[:, None]).astype(np.float32)
    lo, hi = float(d.min()), float(d.max())
    if hi - lo > 1e-6:
        sc = 1.0 / (hi - lo)
        d = (d.astype(np.float64) * np.float64(np.float32(sc)) + np.float64(np.float32(-lo * sc))).astype(np.float32)
    return d
