"""Time the end-to-end tracking loop (vs_slam: batched SuperPoint extraction + Slam::process_frame
per frame, every arithmetic stage on the GPU) on the closed-loop synthetic RGB-D sequence, and
print per-stage device time.  Usage: python tools/bench_tracker.py [--frames 126] [--batch 32]
[--steps 8] [--warmup 2]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=126)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    import torch

    import ate
    import synth
    import vslam_abi
    t0 = time.time()
    L = synth.loop_sequence(a.frames)
    print(f"rendered {a.frames} frames in {time.time() - t0:.1f} s", flush=True)
    U, B = a.frames, a.batch
    dev = torch.device("cuda", 0)
    wrap = np.concatenate([np.arange(U), np.arange(B)])
    bgr = torch.from_numpy(L["bgr"][wrap]).to(dev)
    dep = torch.from_numpy(L["depth"][wrap]).to(dev)
    hdep = [L["depth"][i] for i in wrap]
    ctx = vslam_abi.Context(0)
    S = vslam_abi.Slam(ctx, max_batch=B)

    def step(k):
        g0 = k * B
        i0 = g0 % U
        ts = [1311868164.0 + 0.1 * (g0 + j) for j in range(B)]
        ids = [3 * (g0 + j) for j in range(B)]
        return S.process_batch_dev(B, bgr[i0].data_ptr(), dep[i0].data_ptr(), hdep[i0:i0 + B], ts, ids)

    for k in range(a.warmup):
        step(k)
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    done = 0
    for k in range(a.warmup, a.warmup + a.steps):
        done += int(step(k).sum())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    prof = ctx.profile_read()
    S.finish()
    ids, ts, R, t = S.trajectory()
    g = np.array([(ts_i - 1311868164.0) / 0.1 for ts_i in ts]).round().astype(int) % U
    res = ate.compute_ate(ts, t, ts, L["t_wc"][g])
    frames = a.steps * B
    out = dict(frames_per_s=frames / el, ms_per_frame=el / frames * 1e3, processed=done, frames=frames,
               ate_rmse=res["ate_rmse"], ate_scale=res["scale"], stats=S.stats_dict(),
               stage_ms_per_frame={k: round(v[0] / frames, 4) for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])},
               stage_launches={k: v[1] for k, v in prof.items()})
    print(json.dumps(out), flush=True)
    S.close()
    ctx.close()


if __name__ == "__main__":
    main()
