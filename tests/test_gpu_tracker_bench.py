"""GPU parity of the tracking loop at the bench's own settings (SURVEY.md 8(f)
F1: Slam::process_frame, reference src/Slam.cpp:809-1135, restated in host/tracker.hpp).

bench.py runs vs_slam_process_batch_dev with B = 32 frames per call, each batch's extraction
prefetched behind the previous batch's (vs_slam_prefetch_batch_dev), the default extraction chunk
schedule (even chunks of 8: 8, 8, 8, 8) on its own CU-masked stream, the speculative next-frame chain and the
default VS_SLAM_TRACK_CUS, over the 126-frame closed loop replayed with continuing timestamps.  This test runs exactly that for
the bench's 800 frames (6.3 laps, map past 30k points, 200+ keyframes so that loop closure runs,
Slam.cpp:1084-1086) and the oracle tracker (oracle/orc_slam.cpp: the same control
flow over the CPU restatements) on the same GPU features, and compares decision counters, the whole
trajectory and the map bit for bit: every stage is bit-exact against its CPU restatement, and the
fp64 transcendental functions both sides use (Rodrigues, the 7-point cubic, RANSACUpdateNumIters)
are the correctly rounded ones (csrc/cr_math.h: double-double on the device, libquadmath in the
oracle), so nothing drifts even after hundreds of frames (tools/debug_tracker_divergence.py --loop
416 --tol 0 reports no differing frame)."""
import numpy as np
import pytest
import torch

import ate
import synth
import vslam_abi

pytestmark = pytest.mark.gpu

LOOP = 126
B = 32
STEPS = 25          # 800 frames, as bench.py
T0 = 1311868164.0


@pytest.fixture(scope="module")
def loop():
    return synth.loop_sequence(LOOP, workers=8)


@pytest.fixture(scope="module")
def loop_feats(vsctx, loop):
    out = []
    for i in range(0, LOOP, 32):
        out += vsctx.extract_batch(list(loop["bgr"][i:i + 32]))
    return out


@pytest.fixture(scope="module")
def gpu_run(vsctx, loop):
    dev = torch.device("cuda", 0)
    wrap = np.concatenate([np.arange(LOOP), np.arange(B)])
    bgr = torch.from_numpy(loop["bgr"][wrap]).to(dev)
    dep = torch.from_numpy(loop["depth"][wrap]).to(dev)
    hdep = [loop["depth"][i] for i in wrap]
    torch.cuda.synchronize()
    with vslam_abi.Slam(vsctx, max_batch=B) as S:
        done = []
        for k in range(STEPS):
            g0 = k * B
            i0 = g0 % LOOP
            if k + 1 < STEPS:  # as bench.py: the next batch extracted behind this one
                i1 = (g0 + B) % LOOP
                S.prefetch_batch_dev(B, bgr[i1].data_ptr(), dep[i1].data_ptr())
            done += S.process_batch_dev(B, bgr[i0].data_ptr(), dep[i0].data_ptr(), hdep[i0:i0 + B],
                                        [T0 + 0.1 * (g0 + j) for j in range(B)],
                                        [3 * (g0 + j) for j in range(B)]).tolist()
        traj_raw = S.trajectory()
        S.finish()
        out = done, S.stats(), traj_raw, S.trajectory(), S.map_points(), S.loops()
        n_pgo = S.run_posthoc_pgo()  # Slam::run_posthoc_pgo over the found loop(s)
        return out + ((n_pgo, S.trajectory(), S.map_points()),)


@pytest.fixture(scope="module")
def oracle_run(oracle, loop, loop_feats):
    S = oracle.Slam()
    done = []
    for g in range(STEPS * B):
        k, d = loop_feats[g % LOOP]
        done.append(S.process(k, d, loop["depth"][g % LOOP], T0 + 0.1 * g, 3 * g))
    traj_raw = S.trajectory()
    S.finish()
    out = done, S.stats(), traj_raw, S.trajectory(), S.map_points(), S.loops()
    n_pgo = S.run_posthoc_pgo()
    out = out + ((n_pgo, S.trajectory(), S.map_points()),)
    S.close()
    return out


def test_bench_scale_tracker_matches_oracle(gpu_run, oracle_run, loop):
    g, o = gpu_run, oracle_run
    stats = dict(zip(vslam_abi.SLAM_STATS, g[1].tolist()))
    ostats = dict(zip(vslam_abi.SLAM_STATS, o[1].tolist()))
    assert g[0] == o[0]
    assert stats == ostats, (stats, ostats)
    assert stats["processed"] == STEPS * B
    assert stats["map_points"] > 20000, stats
    for (gi, gts, gR, gt), (oi, ots, oR, ot) in [(g[2], o[2]), (g[3], o[3])]:
        assert np.array_equal(gi, oi) and np.array_equal(gts, ots)
        assert np.array_equal(gR, oR) and np.array_equal(gt, ot)
    (gp, gv), (op, ov) = g[4], o[4]
    assert np.array_equal(gv, ov) and np.array_equal(gp, op)


def test_bench_scale_loop_closure_matches_oracle(gpu_run, oracle_run):
    """LoopCloser::detect + Slam::handle_loop_closure (LoopCloser.cpp:16-100, Slam.cpp:730-798) at
    keyframe 200: the batched candidate evaluation on the GPU (one match launch over every 5th
    keyframe 200+ ids back, one E-RANSAC launch) finds the same loop as the oracle's sequential
    loop, and the PnP-verified constraint is identical bit for bit.  The synthetic sequence is a
    closed loop, so a loop must be found."""
    (ge, gc), (oe, oc) = gpu_run[5], oracle_run[5]
    stats = dict(zip(vslam_abi.SLAM_STATS, gpu_run[1].tolist()))
    assert stats["keyframe_count"] >= 200 and stats["loop_count"] >= 1, stats
    assert np.array_equal(ge, oe) and ge.shape[0] == stats["loop_count"]
    assert np.array_equal(gc.view(np.uint64), oc.view(np.uint64))
    for e in ge:
        assert e[1] - e[0] >= 200  # LC_MIN_FRAME_GAP in frame ids


def test_bench_scale_posthoc_pgo_matches_oracle(gpu_run, oracle_run):
    """Slam::run_posthoc_pgo (Slam.cpp:1748-1755 -> Optimizer.cpp:654-863) over the bench run's
    keyframes and verified loop constraint(s): the GPU pose graph (block-skyline LM) and the
    oracle's dense one give the same keyframe / frame poses and map points to 1e-7 (numeric-Jacobian
noise, tests/test_gpu_pgo.py)."""
    (gn, (gi, _, gR, gt), (gp, gv)), (on, (oi, _, oR, ot), (op, ov)) = gpu_run[6], oracle_run[6]
    assert gn == on
    assert np.array_equal(gi, oi) and np.array_equal(gv, ov)
    assert np.abs(gR - oR).max() < 1e-7 and np.abs(gt - ot).max() < 1e-7
    assert np.abs(gp - op).max() < 1e-6  # map points up to ~10 m from their keyframe
    if gn:  # a loop constraint moved the trajectory
        assert np.abs(gt - gpu_run[3][3]).max() > 1e-6


def test_bench_scale_ate_is_the_algorithms(gpu_run, oracle_run, loop):
    """The ATE and sim(3) scale of the bench sequence are properties of the restated algorithm
    (random SuperPoint weights), not of the GPU path: both trackers give the same numbers."""
    res = []
    for run in (gpu_run, oracle_run):
        ids, ts, R, t = run[3]
        gi = np.round((ts - T0) / 0.1).astype(int) % LOOP
        res.append(ate.compute_ate(ts, t, ts, loop["t_wc"][gi]))
    assert res[0]["ate_rmse"] == res[1]["ate_rmse"] and res[0]["scale"] == res[1]["scale"], res


def test_stale_prefetch_is_discarded(vsctx, loop):
    """A prefetch hint whose buffers the next call does not use is waited for and dropped: the run
    equals one without hints (and the region it held is reused correctly afterwards)."""
    dev = torch.device("cuda", 0)
    Bs = 16
    bgr = torch.from_numpy(loop["bgr"][:4 * Bs]).to(dev)
    dep = torch.from_numpy(loop["depth"][:4 * Bs]).to(dev)
    other = bgr.clone()
    res = []
    for hints in (False, True):
        with vslam_abi.Slam(vsctx, max_batch=Bs) as S:
            for k in range(4):
                g0 = k * Bs
                if hints and k == 1:  # a hint for buffers the next call will not pass
                    S.prefetch_batch_dev(Bs, other[g0 + Bs].data_ptr(), dep[g0 + Bs].data_ptr())
                if hints and k == 2:  # a matching hint
                    S.prefetch_batch_dev(Bs, bgr[g0 + Bs].data_ptr(), dep[g0 + Bs].data_ptr())
                S.process_batch_dev(Bs, bgr[g0].data_ptr(), dep[g0].data_ptr(), list(loop["depth"][g0:g0 + Bs]),
                                    [T0 + 0.1 * (g0 + j) for j in range(Bs)], [3 * (g0 + j) for j in range(Bs)])
            S.finish()
            res.append((S.stats(), S.trajectory(), S.map_points()))
    assert np.array_equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert np.array_equal(a, b)
    for a, b in zip(res[0][2], res[1][2]):
        assert np.array_equal(a, b)
