"""Per-frame divergence between the GPU tracker and the oracle tracker: after every frame, the max
|pose difference| over the trajectory so far, the max map-point difference and the stats that
differ.  Debugging aid.

    python tools/debug_tracker_divergence.py [N]               test_gpu_tracker.py's sequence
    python tools/debug_tracker_divergence.py --loop N [--batch B]  bench.py's closed loop (replayed)

With --loop only the frames around the first divergence are printed."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("visual-slam-pipeline_amd/python", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))

T0 = 1311868164.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", nargs="?", type=int, default=30)
    ap.add_argument("--loop", type=int, default=0)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--after", type=int, default=6, help="frames printed after the first divergence")
    ap.add_argument("--tol", type=float, default=1e-6, help="pose / map difference counted as divergence")
    ap.add_argument("--dump", default=None, help="npz of both trackers' state at the first divergence")
    ap.add_argument("--trace", default=None, help="prefix: write both trackers' stage traces and diff them")
    a = ap.parse_args()
    if a.trace:
        os.environ["VS_TRACE_GPU"] = a.trace + ".gpu.txt"
        os.environ["VS_TRACE_ORACLE"] = a.trace + ".oracle.txt"
    import oracle_py
    import synth
    import vslam_abi
    ctx = vslam_abi.Context(0)
    if a.loop:
        L = synth.loop_sequence(126, workers=8)
        uniq = []
        for i in range(0, 126, 32):
            uniq += ctx.extract_batch(list(L["bgr"][i:i + 32]))
        frames = [(uniq[g % 126], L["depth"][g % 126], T0 + 0.1 * g) for g in range(a.loop)]
    else:
        seq = synth.sequence(a.n)
        feats = []
        for i in range(0, a.n, 8):
            feats += ctx.extract_batch([f["bgr"] for f in seq[i:i + 8]])
        frames = [(k, f["depth"], f["timestamp"]) for f, k in zip(seq, feats)]
    G = vslam_abi.Slam(ctx, max_batch=a.batch)
    O = oracle_py.Slam()
    first = None
    for i, ((k, d), depth, ts) in enumerate(frames):
        rg = G.process_features(k, d, depth, ts, 3 * i)
        ro = O.process(k, d, depth, ts, 3 * i)
        _, _, gR, gt = G.trajectory()
        _, _, oR, ot = O.trajectory()
        gs, os_ = G.stats(), O.stats()
        dR = float(np.max(np.abs(gR - oR))) if len(gR) == len(oR) else -1
        dt = float(np.max(np.abs(gt - ot))) if len(gt) == len(ot) else -1
        gp, gv = G.map_points()
        op, ov = O.map_points()
        dp = float(np.max(np.abs(gp - op), initial=0.0)) if gp.shape == op.shape else -1
        dv = int(np.sum(gv != ov)) if gv.shape == ov.shape else -1
        diff = {vslam_abi.SLAM_STATS[j]: (int(gs[j]), int(os_[j])) for j in range(len(vslam_abi.SLAM_STATS))
                if gs[j] != os_[j]}
        bad = rg != ro or diff or dR > a.tol or dt > a.tol or dp > a.tol or dv != 0 or dR < 0 or dt < 0 or dp < 0
        if bad and first is None:
            first = i
        if not a.loop or (first is not None and i < first + a.after) or i % 50 == 0:
            print(f"frame {i:3d} dR {dR:.3e} dt {dt:.3e} dmap {dp:.3e} dvalid {dv} n_mp {len(gp)}/{len(op)} "
                  f"kf {gs[9]} stats_diff {diff}", flush=True)
        if a.dump and first == i:
            np.savez(a.dump, frame=i, gR=gR, gt=gt, oR=oR, ot=ot, gp=gp, op=op, gv=gv, ov=ov, gs=gs, os=os_)
        if a.loop and first is not None and i >= first + a.after:
            break
    print(f"first divergence at frame {first}", flush=True)
    G.close()
    O.close()
    ctx.close()
    if a.trace:
        diff_traces(a.trace + ".gpu.txt", a.trace + ".oracle.txt")


def diff_traces(pg, po):
    """First differing line of each trace record kind (chain / r3d / rE / motion+ekf / tlm / pnp /
    refined), and the first differing line overall."""
    import re
    g = open(pg).read().splitlines()
    o = open(po).read().splitlines()
    norm = lambda x: re.sub(r"raw=\d+ ", "", x)  # the oracle back end does not report n_raw
    seen = set()
    for k, (x, y) in enumerate(zip(g, o)):
        if norm(x) == norm(y):
            continue
        kind = x.split()[1] if x.split()[0].lstrip("-").isdigit() else x.split()[0]
        if kind in seen:
            continue
        seen.add(kind)
        print(f"first differing '{kind}' line {k}:\n  gpu    {x}\n  oracle {y}")
    if not seen:
        print(f"traces equal over {min(len(g), len(o))} lines")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "--diff":
    diff_traces(sys.argv[2], sys.argv[3])
    sys.exit(0)


if __name__ == "__main__":
    main()
