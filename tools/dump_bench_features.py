"""Dump the SuperPoint features of bench.py's closed-loop sequence (the 126 unique frames of one lap,
extracted by libvslam_hip.so on the GPU) so the tracker's behaviour on the headline's own input can be
replayed on the CPU through the oracle tracker (GPU tracker == oracle tracker bit for bit,
tests/test_gpu_tracker_bench.py).  Debugging aid.

    python tools/dump_bench_features.py gpurun_out/bench_features.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))


def main():
    import synth
    import vslam_abi
    out = sys.argv[1]
    L = synth.loop_sequence(126, workers=8)
    kps = np.zeros((126, 400), vslam_abi.KEYPOINT_DTYPE)
    desc = np.zeros((126, 400, 256), np.float32)
    n = np.zeros(126, np.int32)
    with vslam_abi.Context(0) as ctx:
        for i in range(0, 126, 32):
            for j, (k, d) in enumerate(ctx.extract_batch(list(L["bgr"][i:i + 32]))):
                n[i + j] = len(k)
                kps[i + j, :len(k)] = k
                desc[i + j, :len(k)] = d
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    np.savez_compressed(out, kps=kps, desc=desc, n=n)
    print(f"{out}: {n.sum()} keypoints over 126 frames")


if __name__ == "__main__":
    main()
