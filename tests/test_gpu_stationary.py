"""The stationary / accelerometer branch of Slam::process_frame (reference src/Slam.cpp:615-694
process_stationary_frame, :912-951 the post-stationary transition, :1580-1651 accelerometer data,
gravity direction and is_frame_stationary; restated in host/tracker.hpp) on the GPU tracker against
the oracle tracker: a drive that stops for 12 frames and continues (synth.stationary_sequence, with
a 100 Hz accelerometer stream whose vibration drops while the camera is held) through
vs_slam_process_batch_dev and through the oracle on the same features.  Counters, trajectory and
map bit for bit; the branch is exercised (stationary frames counted, the transition recomputes the
motion, the gravity height prior is active)."""
import numpy as np
import pytest
import torch

import synth
import vslam_abi

pytestmark = pytest.mark.gpu

T0 = 1311868164.0


@pytest.fixture(scope="module")
def seq():
    return synth.stationary_sequence(workers=8)


def test_stationary_branch_matches_oracle(vsctx, oracle, seq):
    n = len(seq["bgr"])
    B = 19
    assert n % B == 0
    ts = T0 + seq["timestamps"]
    ids = [3 * g for g in range(n)]
    acc = seq["accel"].copy()
    acc[:, 0] += T0
    dev = torch.device("cuda", 0)
    bgr = torch.from_numpy(seq["bgr"]).to(dev)
    dep = torch.from_numpy(seq["depth"]).to(dev)
    torch.cuda.synchronize()
    with vslam_abi.Slam(vsctx, max_batch=B) as S:
        S.set_initial_pose(np.eye(3), np.zeros(3))
        S.set_accelerometer(acc)
        for i0 in range(0, n, B):
            S.process_batch_dev(B, bgr[i0].data_ptr(), dep[i0].data_ptr(), list(seq["depth"][i0:i0 + B]),
                                list(ts[i0:i0 + B]), ids[i0:i0 + B])
        S.finish()
        g = (S.stats(), S.trajectory(), S.map_points())
    feats = []
    for i0 in range(0, n, B):
        feats += vsctx.extract_batch(list(seq["bgr"][i0:i0 + B]))
    O = oracle.Slam()
    O.set_initial_pose(np.eye(3), np.zeros(3))
    O.set_accelerometer(acc)
    for k in range(n):
        O.process(feats[k][0], feats[k][1], seq["depth"][k], ts[k], ids[k])
    O.finish()
    o = (O.stats(), O.trajectory(), O.map_points())
    O.close()
    st = dict(zip(vslam_abi.SLAM_STATS, g[0].tolist()))
    assert np.array_equal(g[0], o[0]), (st, dict(zip(vslam_abi.SLAM_STATS, o[0].tolist())))
    assert st["stationary"] >= 8, st          # held frames after the first 5 (frame_count_ > 5)
    assert st["chains_recomputed"] >= 1, st   # :916-951 motion recomputed after the stop
    for a, b in zip(g[1], o[1]):
        assert np.array_equal(a, b)
    for a, b in zip(g[2], o[2]):
        assert np.array_equal(a, b)
