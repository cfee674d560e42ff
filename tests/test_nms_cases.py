"""The long-chain NMS heatmaps of tests/nms_cases.py decode as intended (oracle decode, the
reference's softmax restatement), and the oracle's sequential greedy NMS gives the structure the
GPU tests rely on (CPU only)."""
import numpy as np

import nms_cases


def test_serpentine_scores_fall_along_the_chain(oracle):
    semi, n = nms_cases.serpentine_semi()
    heat = oracle.decode_heatmap(semi)
    pts = nms_cases.serpentine_path()
    assert n == len(pts) > 4500
    s = np.array([heat[y, x] for x, y in pts])
    assert np.all(np.diff(s) < 0) and s[-1] > 0.005
    mask = np.zeros_like(heat, bool)
    for x, y in pts:
        mask[y, x] = True
    assert np.all(heat[~mask] <= 0.005)
    for a, b in zip(pts, pts[1:]):  # consecutive chain pixels share a 9 x 9 window
        assert max(abs(a[0] - b[0]), abs(a[1] - b[1])) <= 4


def test_serpentine_greedy_keeps_every_other_chain_pixel(oracle):
    semi, _ = nms_cases.serpentine_semi()
    dg = np.ones((256, 60, 80), np.float32) / 16.0
    kps, _ = oracle.postprocess(semi, dg, order_mode=1)
    assert len(kps) == 400
    assert np.array_equal(kps["x"][:80], np.arange(0, 640, 8)) and np.all(kps["y"][:80] == 2)


def test_gradient_is_above_threshold_everywhere_and_falls_in_raster_order(oracle):
    heat = oracle.decode_heatmap(nms_cases.gradient_semi()).reshape(-1)
    assert heat.min() > 0.005
    assert np.mean(np.diff(heat) < 0) > 0.95
