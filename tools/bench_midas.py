"""MiDaS v2.1-small network alone on the whole chip (vs_midas_forward_dev, B frames of 256x256x3):
ms per batch over --reps launches after a warm-up; run under rocprofv3 --kernel-trace --stats for the
per-kernel split (k_mid_conv 1x1 / strided, k_wino3 stride-1 3x3, k_mid_dw, k_mid_up).
Usage: python tools/bench_midas.py [--batch 32] [--reps 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))

import torch  # noqa: E402

import vslam_abi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    with vslam_abi.Context(0) as ctx:
        m = vslam_abi.Midas(ctx)
        x = torch.from_numpy(rng.standard_normal((a.batch, 256, 256, 3)).astype(np.float32)).to(dev)
        y = torch.zeros((a.batch, 256, 256), dtype=torch.float32, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(3):
            m.forward_dev(a.batch, x.data_ptr(), y.data_ptr(), s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            m.forward_dev(a.batch, x.data_ptr(), y.data_ptr(), s)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.reps
        fl = vslam_abi.Midas.flops_per_frame() * a.batch
        print(json.dumps({"batch": a.batch, "ms_per_batch": round(ms, 4), "ms_per_frame": round(ms / a.batch, 5),
                          "tflops": round(fl / ms / 1e9, 2), "frac": round(fl / ms / 1e9 / 157.3, 4)}))
        m.close()


if __name__ == "__main__":
    main()
