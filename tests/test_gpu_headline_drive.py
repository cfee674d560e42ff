"""Parity of the headline's own input: the tracking loop (SURVEY.md 8(f) F1,
Slam::process_frame, reference src/Slam.cpp:809-1135; main.cpp:1096-1107 the frame loop) on exactly the
drive and schedule bench.py times with the driver's command (--steps 20 --warmup 5, B = 32):
synth.pioneer_trajectory(928) — the non-repeating Pioneer-like drive, every processed frame distinct —
through vs_slam_process_batch_dev in bench.headline_plan's ranges (5 warm-up steps, the 20 timed steps
= frames 160-799, 4 stage-profiled steps), each range prefetching its next batch
(bench.run_tracker_steps), the default extraction chunks, CU sets and speculative chain, the dense
fusion attached and the bench's HIP-event profiling toggled as it toggles it.

Against it: (1) the oracle tracker (oracle/orc_slam.cpp, the same control flow over the CPU
restatements) on the same GPU features — per-frame results, decision counters, the raw and the
RTS-smoothed trajectory, the map and the loop edges / constraints bit for bit; (2) the oracle run's op
log replayed through tests/slam_glue_ref.py, the numpy restatement of the glue that shares no source
with host/tracker.hpp, which makes every per-frame decision itself.  The frames-per-second line is
therefore a rate of a computation whose every decision is pinned."""
import os

import numpy as np
import pytest
import torch

import bench
import slam_glue_ref
import synth
import vslam_abi

pytestmark = pytest.mark.gpu

B, WARMUP, STEPS, PROFILE_STEPS = 32, 5, 20, 4   # the driver's command and bench.py's defaults
T0 = bench.T0


@pytest.fixture(scope="module")
def drive():
    n_path, ranges = bench.headline_plan(B, WARMUP, STEPS, PROFILE_STEPS)
    assert n_path == 928 and ranges == [(0, 5), (5, 25), (25, 29)]
    poses = synth.pioneer_trajectory(n_path)
    bgr, dep = synth.render_frames(poses, list(range(n_path)), workers=min(16, os.cpu_count() or 1))
    return n_path, ranges, bgr, dep


@pytest.fixture(scope="module")
def gpu_run(vsctx, drive):
    n_path, ranges, bgr_h, dep_h = drive
    dev = torch.device("cuda", 0)
    bgr = torch.from_numpy(bgr_h).to(dev)
    dep = torch.from_numpy(dep_h).to(dev)
    hdep = [dep_h[i] for i in range(n_path)]
    torch.cuda.synchronize()
    dense = vslam_abi.Dense(vsctx)
    with vslam_abi.Slam(vsctx, max_batch=B) as S:
        S.attach_dense(dense)
        done = bench.run_tracker_steps(S, bgr, dep, hdep, B, *ranges[0])
        torch.cuda.synchronize()
        vsctx.profile(2)      # bench: the network stages' events during the timed steps
        vsctx.profile_reset()
        done += bench.run_tracker_steps(S, bgr, dep, hdep, B, *ranges[1])
        torch.cuda.synchronize()
        vsctx.profile(True)   # bench: every stage's events during the profiled steps
        vsctx.profile_reset()
        done += bench.run_tracker_steps(S, bgr, dep, hdep, B, *ranges[2])
        torch.cuda.synchronize()
        vsctx.profile(False)
        traj_raw = S.trajectory()
        S.finish()
        out = dict(done=[bool(x) for x in done], stats=S.stats(), traj_raw=traj_raw, traj=S.trajectory(),
                   map=S.map_points(), loops=S.loops(), dense=dense.size())
    dense.close()
    del bgr, dep
    return out


@pytest.fixture(scope="module")
def oracle_run(vsctx, oracle, drive, tmp_path_factory):
    n_path, ranges, bgr_h, dep_h = drive
    feats = []
    for i in range(0, n_path, B):
        feats += vsctx.extract_batch(list(bgr_h[i:i + B]))
    n_track = ranges[-1][1] * B
    log = str(tmp_path_factory.mktemp("oplog") / "headline.jsonl")
    os.environ["VS_OPLOG"] = log
    try:
        S = oracle.Slam()
    finally:
        del os.environ["VS_OPLOG"]
    done = []
    for g in range(n_track):
        k, d = feats[g]
        done.append(bool(S.process(k, d, dep_h[g], T0 + 0.1 * g, 3 * g)))
    traj_raw = S.trajectory()
    S.finish()
    out = dict(done=done, stats=S.stats(), traj_raw=traj_raw, traj=S.trajectory(), map=S.map_points(),
               loops=S.loops(), log=log, feats=feats[:n_track])
    S.close()  # flushes the op log
    return out


def test_headline_drive_tracker_matches_oracle(gpu_run, oracle_run):
    g, o = gpu_run, oracle_run
    stats = dict(zip(vslam_abi.SLAM_STATS, g["stats"].tolist()))
    ostats = dict(zip(vslam_abi.SLAM_STATS, o["stats"].tolist()))
    print(stats)
    assert g["done"] == o["done"]
    assert stats == ostats, (stats, ostats)
    assert len(g["done"]) == 29 * B
    assert stats["map_points"] > 20000 and stats["keyframes"] > 200, stats   # keyframe 200: loop check ran
    for key in ("traj_raw", "traj"):
        for a, b in zip(g[key], o[key]):
            assert np.array_equal(a, b), key
    (gp, gv), (op, ov) = g["map"], o["map"]
    assert np.array_equal(gv, ov) and np.array_equal(gp, op)
    (ge, gc), (oe, oc) = g["loops"], o["loops"]
    assert np.array_equal(ge, oe) and np.array_equal(gc.view(np.uint64), oc.view(np.uint64))
    assert g["dense"] > 0


def test_headline_drive_glue_replays_independently(oracle_run, drive):
    """The oracle's op log of the same drive through the numpy glue restatement: every frame's branch,
    keyframe flag, pose (<= 1e-9), map appends, visibility flags, PnP inputs and the loop check at
    keyframe 200 are its own decisions; the run's counters equal the C++ glue's."""
    n_path, ranges, bgr_h, dep_h = drive
    o = oracle_run
    G = slam_glue_ref.GlueRef(o["log"])
    for g, (k, d) in enumerate(o["feats"]):
        G.process_frame(slam_glue_ref.Frame(3 * g, T0 + 0.1 * g, k, dep_h[g]))
    st = dict(zip(vslam_abi.SLAM_STATS, o["stats"].tolist()))
    for key in ("via_3d3d", "via_emat", "emat_failed", "bridges", "recoveries", "recovery_failed", "pnp_refined",
                "periodic_pnp", "triangulated", "depth_points", "culled", "stationary"):
        assert st[key] == G.counts[key], (key, st[key], G.counts[key])
    assert st["keyframes"] == G.keyframe_count and st["map_points"] == len(G.mp_pos)
    assert st["map_valid"] == G._n_valid() and st["loop_count"] == G.loop_count
    edges, cons = o["loops"]
    assert [tuple(e) for e in edges.tolist()] == G.loop_edges
    assert len(cons) == len(G.loop_constraints)
    print({b: sum(1 for x in G.branch.values() if x == b) for b in sorted(set(G.branch.values()))}, G.counts)
