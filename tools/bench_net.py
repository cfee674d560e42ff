"""SuperPoint network alone on the whole chip: per-layer device time (HIP events on the launch
stream, vs_profile_enable) and TFLOP/s at 8 and 32 frames per launch.  Library under test:
VS_LIB_PATH (another build of libvslam_hip.so, for same-box kernel A/B), default the in-tree one.
Prints one JSON line.  Usage: python tools/bench_net.py [--reps 10] [--tag NAME]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import vslam_abi  # noqa: E402
from bench import LAYER_FLOPS, FP32_MFMA_PEAK_TFLOPS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tag", default=os.environ.get("VS_LIB_PATH", "in-tree"))
    ap.add_argument("--frames", default="8,32")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    H, W = 480, 640
    rng = np.random.default_rng(3)
    out = {"tag": args.tag, "peak_tflops": FP32_MFMA_PEAK_TFLOPS}
    with vslam_abi.Context(0) as ctx:
        for nb in [int(x) for x in args.frames.split(",")]:
            bgr = torch.from_numpy(rng.integers(0, 256, (nb, H, W, 3), dtype=np.uint8)).to(dev)
            semi = torch.zeros((nb, 60, 80, vslam_abi.SEMI_CH), dtype=torch.float32, device=dev)
            dg = torch.zeros((nb, 60, 80, vslam_abi.DESC_DIM), dtype=torch.float32, device=dev)
            s = torch.cuda.current_stream().cuda_stream
            for _ in range(3):
                ctx.network_batch_dev(nb, bgr.data_ptr(), H, W, semi.data_ptr(), dg.data_ptr(), s)
            torch.cuda.synchronize()
            ctx.profile(True)
            ctx.profile_reset()
            for _ in range(args.reps):
                ctx.network_batch_dev(nb, bgr.data_ptr(), H, W, semi.data_ptr(), dg.data_ptr(), s)
            torch.cuda.synchronize()
            prof = ctx.profile_read()
            ctx.profile(False)
            layers, tot_ms, tot_fl = {}, 0.0, 0.0
            for k, (ms, n) in prof.items():
                if not n:
                    continue
                per = ms / n
                e = {"ms_per_launch": round(per, 4)}
                if k in LAYER_FLOPS:
                    tf = LAYER_FLOPS[k] * nb / (per / 1e3) / 1e12
                    e.update(tflops=round(tf, 2), frac=round(tf / FP32_MFMA_PEAK_TFLOPS, 4))
                    tot_fl += LAYER_FLOPS[k] * nb * n
                tot_ms += ms
                layers[k] = e
            out[f"frames_{nb}"] = {"layers": layers, "network_ms_per_launch": round(tot_ms / args.reps, 4),
                                   "network_tflops": round(tot_fl / (tot_ms / 1e3) / 1e12, 2)}
            del bgr, semi, dg
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
