"""Descriptor-match kernel against its roofline (north star: "descriptor-match kernel
... in rocprof"): vs_match_pairs_dev (Slam::match_features, Slam.cpp:1140-1172: 2-NN L2 + ratio
test) over P consecutive frame pairs per launch, n x n keypoints, 256-d fp32 descriptors.

    python tools/bench_match.py [--n 400] [--reps 20] [--pairs 1,8,32,128,512]

Per pair the algorithmic work is 2 n^2 256 FLOP (the distance matrix) and 2 n 256 4 bytes of
descriptors (each frame read once per pair it is in).  The time is the library's HIP-event stage
"match" (k_match + k_match_compact, events on the stream the kernels run on).  Prints one JSON line
per P with TFLOP/s and GB/s against the fp32 MFMA and HBM peaks (MI355X_MICROARCH.md)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))

FP32_MFMA_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pairs", default="1,8,32,128,512")
    args = ap.parse_args()
    import torch

    import vslam_abi as va
    ctx = va.Context(0)
    n, cap = args.n, va.SP_MAX_KEYPOINTS
    assert 0 < n <= cap
    s = torch.cuda.current_stream().cuda_stream
    for P in [int(x) for x in args.pairs.split(",")]:
        F = P + 1
        g = torch.Generator(device="cuda").manual_seed(P)
        desc = torch.randn(F, cap, 256, device="cuda", generator=g)
        desc = desc / desc.norm(dim=2, keepdim=True)
        nn = torch.full((F,), n, dtype=torch.int32, device="cuda")
        pairs = torch.tensor([[p, p + 1] for p in range(P)], dtype=torch.int32, device="cuda")
        raw = torch.zeros(P * cap * 16, dtype=torch.uint8, device="cuda")
        good = torch.zeros_like(raw)
        nraw = torch.zeros(P, dtype=torch.int32, device="cuda")
        ngood = torch.zeros_like(nraw)

        def run():
            ctx.match_pairs_dev(P, pairs.data_ptr(), F, desc.data_ptr(), nn.data_ptr(), cap, 0.75, raw.data_ptr(),
                                nraw.data_ptr(), good.data_ptr(), ngood.data_ptr(), s)
        run()
        torch.cuda.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        for _ in range(args.reps):
            run()
        torch.cuda.synchronize()
        ms, launches = ctx.profile_read()["match"]
        ctx.profile(False)
        t = ms / launches / 1e3
        flops = 2.0 * n * n * 256 * P
        bytes_ = 2.0 * n * 256 * 4 * P
        print(json.dumps({"kernel": "match_pairs", "pairs": P, "n": n, "us_per_launch": round(t * 1e6, 2),
                          "tflops": round(flops / t / 1e12, 2),
                          "mfma_frac": round(flops / t / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
                          "gbs": round(bytes_ / t / 1e9, 1), "hbm_frac": round(bytes_ / t / 1e9 / HBM_PEAK_GBS, 4),
                          "pairs_per_s": round(P / t, 1), "ngood_mean": float(ngood.float().mean())}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
