"""Host side of the monocular stream (BASELINE config[4]): the HD camera of the synthetic renderer and
the scale fallback of the pose chain (Slam.cpp:976-980: last good scale, then MOTION_SCALE)."""
import numpy as np

import synth
from vslam_pipeline import MOTION_SCALE, PoseChain


def test_hd_render_shape_and_depth():
    R, t = synth.loop_trajectory(126)[0]
    bgr, depth = synth._render_one((0, R, t, synth.SEED, synth.K_HD, synth.W_HD, synth.H_HD))
    assert bgr.shape == (720, 1280, 3) and bgr.dtype == np.uint8
    assert depth.shape == (720, 1280) and depth.dtype == np.float32
    assert bgr.std() > 10  # textured


def test_pose_chain_scale_fallback():
    I, z = np.eye(3).reshape(9), np.zeros(3)
    t = np.array([0.0, 0.0, 1.0])
    c = PoseChain()
    _, t1 = c.step(0, I, z, 1, I, t, -1.0)  # no scale yet: MOTION_SCALE
    assert np.allclose(t1, -MOTION_SCALE * t)
    _, t2 = c.step(0, I, z, 1, I, t, 0.2)  # a measured scale is used and remembered
    assert np.allclose(t2 - t1, -0.2 * t)
    _, t3 = c.step(0, I, z, 1, I, t, -1.0)  # then it is the fallback
    assert np.allclose(t3 - t2, -0.2 * t)
    _, t4 = c.step(0, I, z, 0, I, t, -1.0)  # neither estimate: the pose is kept
    assert np.array_equal(t4, t3)
