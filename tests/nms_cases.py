"""Heatmaps whose greedy NMS (reference src/FeatureExtractor.cpp:219-259) has long dependency
chains, built as SuperPoint `semi` logits (65 x hc x wc, channel c = pixel (c // 8, c % 8) of the
cell, 64 = dustbin) so that the decoded heat (softmax per cell) is the intended score up to
float rounding: pixel logits log(h), dustbin log(1 - sum h), total mass 1.

serpentine: one chain of pixels 4 apart snaking along rows 16 apart over the whole frame, scores
strictly decreasing along it.  Each chain pixel's fate depends on its predecessor's, so the
priority-MIS needs about one round per two chain pixels (thousands), and every 32 x 32 NMS tile
border the chain crosses costs one tile round: far beyond the fixed tile-round budget.

gradient: every pixel above threshold with scores falling in raster order; the greedy result is
a lattice whose decisions sweep from the top-left corner, crossing tiles one per round."""
import numpy as np


def _semi_from_heat(target, hc, wc):
    """target: (hc*8, wc*8) float64 scores (0 = no candidate)."""
    t = target.reshape(hc, 8, wc, 8).transpose(1, 3, 0, 2).reshape(64, hc, wc)
    mass = t.sum(axis=0)
    assert mass.max() < 0.999
    semi = np.full((65, hc, wc), -30.0)
    semi[:64][t > 0] = np.log(t[t > 0])
    semi[64] = np.log(1.0 - mass)
    return semi.astype(np.float32)


def serpentine_path(hc=60, wc=80, row_gap=16, step=4):
    H, W = hc * 8, wc * 8
    xs = list(range(0, W - step + 1, step))
    pts = []
    rows = list(range(2, H - 2, row_gap))
    for k, y in enumerate(rows):
        line = xs if k % 2 == 0 else xs[::-1]
        pts += [(x, y) for x in line]
        if k + 1 < len(rows):
            pts += [(line[-1], y + d) for d in range(step, row_gap, step)]
    return pts


def serpentine_semi(hc=60, wc=80, hi=0.24, lo=0.01):
    pts = serpentine_path(hc, wc)
    target = np.zeros((hc * 8, wc * 8))
    for (x, y), h in zip(pts, np.linspace(hi, lo, len(pts))):
        target[y, x] = h
    return _semi_from_heat(target, hc, wc), len(pts)


def gradient_semi(hc=60, wc=80, hi=0.0155, lo=0.006):
    n = hc * 8 * wc * 8
    target = np.linspace(hi, lo, n).reshape(hc * 8, wc * 8)
    return _semi_from_heat(target, hc, wc)
