"""Latency of the RANSAC-style geometry kernels (report us per call and
hypotheses/s) on synthetic problems of the pipeline's sizes.

    python tools/bench_geometry.py [--pairs 32] [--n 300] [--reps 20]

Times vs_fmat_verify_pairs_dev (P frame pairs per launch) and vs_solve_pnp_batch_dev (P problems
per launch) with HIP events on the library's stream, at several outlier fractions, and prints one
JSON line per case with the registrator's iteration counts."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("visual-slam-pipeline_amd/python", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=32)
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch

    import vslam_abi as va
    from test_gpu_fmat import _pairs_inputs
    from test_oracle_fmat import two_view
    from test_oracle_pnp import pnp_problem

    ctx = va.Context(0)

    def timed(fn, stage):
        """Average device time per launch from the library's HIP-event stage profiler (the events
        sit on the stream the kernel runs on)."""
        fn()
        torch.cuda.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        ms, launches = ctx.profile_read()[stage]
        ctx.profile(False)
        return ms / launches

    P, n = args.pairs, args.n
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).cuda()  # noqa: E731
    for out in (0.1, 0.3, 0.5):
        probs = [two_view(n, 1000 + i, 0.7, out)[:2] for i in range(P)]
        cap, pairs, kp_tab, goods, ngood = _pairs_inputs(va, probs)
        d_pairs, d_kps, d_good, d_ngood = dev(pairs), dev(kp_tab), dev(goods), dev(ngood)
        d_F = torch.zeros(P, 9, dtype=torch.float64, device="cuda")
        d_kept = torch.zeros(P * cap * 16, dtype=torch.uint8, device="cuda")
        d_nk = torch.zeros(P, dtype=torch.int32, device="cuda")
        d_err = torch.zeros(P, 2, dtype=torch.float64, device="cuda")
        d_diag = torch.zeros(P, 8, dtype=torch.int32, device="cuda")

        def run():
            ctx.fmat_verify_pairs_dev(P, d_pairs.data_ptr(), d_kps.data_ptr(), cap, d_good.data_ptr(),
                                      d_ngood.data_ptr(), d_F.data_ptr(), d_kept.data_ptr(), d_nk.data_ptr(),
                                      d_err.data_ptr(), d_diag.data_ptr(), torch.cuda.current_stream().cuda_stream)
        ms = timed(run, "fmat_ransac")
        dg = d_diag.cpu().numpy()
        hyp = int(dg[:, 1].sum())
        print(json.dumps({"kernel": "fmat_verify_pairs", "pairs": P, "n": n, "outliers": out,
                          "ms_per_launch": round(ms, 4), "us_per_pair": round(ms * 1e3 / P, 2),
                          "iterations_mean": float(dg[:, 1].mean()), "iterations_max": int(dg[:, 1].max()),
                          "hypotheses_per_s": round(hyp / (ms / 1e3), 1)}), flush=True)

    for out in (0.1, 0.3, 0.5):
        probs = [pnp_problem(n, 2000 + i, noise=0.7, outlier_frac=out) for i in range(P)]
        off = np.cumsum([0] + [len(p[0]) for p in probs]).astype(np.int32)
        obj = torch.from_numpy(np.concatenate([p[0] for p in probs])).cuda()
        img = torch.from_numpy(np.concatenate([p[1] for p in probs])).cuda()
        d_off = torch.from_numpy(off).cuda()
        dR = torch.zeros(P, 9, dtype=torch.float64, device="cuda")
        dt = torch.zeros(P, 3, dtype=torch.float64, device="cuda")
        dstat = torch.zeros(P, 8, dtype=torch.int32, device="cuda")
        dmask = torch.zeros(int(off[-1]), dtype=torch.uint8, device="cuda")

        def runp():
            ctx.solve_pnp_batch_dev(P, obj.data_ptr(), img.data_ptr(), d_off.data_ptr(), 100, 10, dR.data_ptr(),
                                    dt.data_ptr(), dstat.data_ptr(), dmask.data_ptr(),
                                    stream=torch.cuda.current_stream().cuda_stream)
        ms = timed(runp, "solve_pnp")
        st = dstat.cpu().numpy()
        print(json.dumps({"kernel": "solve_pnp_batch", "problems": P, "n": n, "outliers": out, "iters": 100,
                          "ms_per_launch": round(ms, 4), "us_per_problem": round(ms * 1e3 / P, 2),
                          "ransac_iterations_mean": float(st[:, 2].mean()), "lm_iterations_mean": float(st[:, 4].mean()),
                          "success": int(st[:, 0].sum())}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
