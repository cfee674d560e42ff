"""Long-run trajectory quality of the CPU oracle tracker on the bench's closed-loop sequence.

Answers whether the bench's ATE / sim(3)-scale drift over many laps is the
reference algorithm itself (with seeded random SuperPoint weights) or a GPU-vs-oracle divergence:
the oracle tracker (oracle/orc_slam.cpp over the CPU restatements, test infrastructure) runs the
same replayed 126-frame loop with the same timestamps / frame ids as bench.py, and the ATE
(Umeyama sim(3), main.cpp:258-332) is reported at checkpoints.

Features: the oracle's CPU SuperPoint (--features cpu, default) or a .npz written by a GPU run
(--features path.npz with kps_<i> / desc_<i> for the 126 loop frames).

Usage: python tools/oracle_long_run.py [--frames 800] [--features cpu|file.npz] [--out res.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

LOOP = 126
T0 = 1311868164.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=800)
    ap.add_argument("--features", default="cpu")
    ap.add_argument("--cache", default="/tmp/vs_loop_feats_cpu.npz")
    ap.add_argument("--out", default=None)
    ap.add_argument("--checkpoints", default="126,256,384,512,640,800")
    args = ap.parse_args()
    import ate
    import oracle_py as oracle
    import synth

    L = synth.loop_sequence(LOOP, workers=min(8, os.cpu_count() or 1))
    feats = None
    src = args.features if args.features != "cpu" else args.cache
    if os.path.exists(src):
        z = np.load(src)
        feats = [(z[f"kps_{i}"], z[f"desc_{i}"]) for i in range(LOOP)]
    elif args.features == "cpu":
        w = _weights()
        feats = []
        t0 = time.time()
        for i in range(LOOP):
            feats.append(oracle.extract(w, L["bgr"][i], nthreads=os.cpu_count() or 1))
        print(f"extracted {LOOP} frames on the CPU in {time.time() - t0:.1f} s", flush=True)
        np.savez(args.cache, **{f"kps_{i}": k for i, (k, _) in enumerate(feats)},
                 **{f"desc_{i}": d for i, (_, d) in enumerate(feats)})
    else:
        raise SystemExit(f"no features at {src}")

    cps = sorted(int(c) for c in args.checkpoints.split(","))
    S = oracle.Slam()
    res = {"frames": args.frames, "features": args.features, "checkpoints": []}
    t0 = time.time()
    for g in range(args.frames):
        k, d = feats[g % LOOP]
        S.process(k, d, L["depth"][g % LOOP], T0 + 0.1 * g, 3 * g)
        if g + 1 in cps:
            ids, ts, R, t = S.trajectory()
            gi = np.round((ts - T0) / 0.1).astype(int) % LOOP
            a = ate.compute_ate(ts, t, ts, L["t_wc"][gi])
            import vslam_abi
            st = dict(zip(vslam_abi.SLAM_STATS, S.stats().tolist()))
            row = {"frames": g + 1, "ate_rmse_m": round(a["ate_rmse"], 4), "scale": round(a["scale"], 4),
                   "map_points": st.get("map_points"), "keyframes": st.get("keyframes"),
                   "via_3d3d": st.get("via_3d3d"), "elapsed_s": round(time.time() - t0, 1)}
            res["checkpoints"].append(row)
            print(json.dumps(row), flush=True)
    S.finish()
    ids, ts, R, t = S.trajectory()
    gi = np.round((ts - T0) / 0.1).astype(int) % LOOP
    a = ate.compute_ate(ts, t, ts, L["t_wc"][gi])
    res["final_after_rts"] = {"ate_rmse_m": round(a["ate_rmse"], 4), "scale": round(a["scale"], 4)}
    print(json.dumps(res["final_after_rts"]), flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)
    S.close()


LAYERS = [(1, 64, 3), (64, 64, 3), (64, 64, 3), (64, 64, 3), (64, 128, 3), (128, 128, 3), (128, 128, 3),
          (128, 128, 3), (128, 256, 3), (256, 65, 1), (128, 256, 3), (256, 256, 1)]


def _weights(seed=20261015):
    """The product's seeded He-normal weights (vs_ctx.hip synth_weights: splitmix64 -> Box-Muller),
    restated in numpy for a CPU-only run (libm-level differences in log/cos are irrelevant here)."""
    M = (1 << 64) - 1
    st = seed
    total = sum(co * ci * k * k + co for ci, co, k in LAYERS)
    out = np.empty(total, np.float32)
    pos = 0

    def nxt():
        nonlocal st
        st = (st + 0x9E3779B97F4A7C15) & M
        z = st
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)
    import math
    for ci, co, k in LAYERS:
        sd = math.sqrt(2.0 / (ci * k * k))
        for n, scale in ((co * ci * k * k, sd), (co, 0.05)):
            for _ in range(n):
                u1 = ((nxt() >> 11) + 1) * (1.0 / 9007199254740992.0)
                u2 = (nxt() >> 11) * (1.0 / 9007199254740992.0)
                out[pos] = math.sqrt(-2.0 * math.log(u1)) * math.cos(6.283185307179586 * u2) * scale
                pos += 1
    return out


if __name__ == "__main__":
    main()
