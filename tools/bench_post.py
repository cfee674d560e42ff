"""SuperPoint post-processing alone (FeatureExtractor.cpp:126-259 after the network: decode, greedy
NMS with the score floor, top-400, border erase, descriptor sampling) on B synthetic 640x480
frames' network outputs resident in HBM, whole chip, for rocprofv3 kernel traces:

    python tools/bench_post.py [--batch 32] [--reps 20]

Prints one JSON line: ms per frame per stage (HIP events) and the HBM roofline fraction against
SURVEY.md 8(d)'s 4.536 MB per frame."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    import synth
    import vslam_abi as va
    B, H, W, cap = a.batch, 480, 640, va.SP_MAX_KEYPOINTS
    L = synth.loop_sequence(B, workers=8)
    dev = torch.device("cuda", 0)
    ctx = va.Context(0)
    bgr = torch.from_numpy(L["bgr"]).to(dev)
    semi = torch.zeros((B, 60, 80, va.SEMI_CH), dtype=torch.float32, device=dev)
    dg = torch.zeros((B, 60, 80, va.DESC_DIM), dtype=torch.float32, device=dev)
    kps = torch.zeros((B, cap * 28), dtype=torch.uint8, device=dev)
    desc = torch.zeros((B, cap, 256), dtype=torch.float32, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ctx.network_batch_dev(B, bgr.data_ptr(), H, W, semi.data_ptr(), dg.data_ptr(), s)
    run = lambda: ctx.postprocess_batch_dev(B, semi.data_ptr(), dg.data_ptr(), H, W, kps.data_ptr(), desc.data_ptr(),
                                            n.data_ptr(), cap, s)
    run()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(a.reps):
        run()
    torch.cuda.synchronize()
    p = ctx.profile_read()
    st = {k: round(p[k][0] / (a.reps * B), 5) for k in ("decode", "nms_rounds", "nms_select", "sample") if k in p}
    ms = sum(st.values())
    byt = 1248000 + 1638400 + 1228800 + 420800
    print(json.dumps({"batch": B, "reps": a.reps, "ms_per_frame": round(ms, 5), "stage_ms_per_frame": st,
                      "keypoints_per_frame": float(n.float().mean()),
                      "hbm_gbs": round(byt / (ms / 1e3) / 1e9, 1), "hbm_frac": round(byt / (ms / 1e3) / 8e12, 5)}))
    ctx.close()


if __name__ == "__main__":
    main()
