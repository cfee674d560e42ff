"""Throughput of the per-frame hot path on MI355X (BASELINE.json metric, config[1] workload).

One "step" = B consecutive processed 640x480 RGB-D frames per GPU, already resident in HBM, pushed
through the whole per-frame hot path by libvslam_hip.so:
    FeatureExtractor::extract   (SuperPoint fp32 network + decode + greedy NMS + descriptor sampling)
    Slam::match_features        (exact 2-NN + 0.75 ratio test, frame i-1 -> frame i)
    F-matrix verification       (findFundamentalMat(FM_RANSAC, 3.0, 0.999) + ordered filtering)
    Slam::estimate_motion_3d3d  (200-iteration 3D-3D RANSAC + refit, on the F-filtered matches)
    Slam::estimate_motion       (5-point essential matrix + recoverPose + depth scale, for the pairs
                                 whose 3D-3D estimate failed, Slam.cpp:965-984)
plus the host pose chain on the returned (R, t) (Slam.cpp:963-964).  Steps are software-pipelined
over two HIP streams (DevicePipeline): step i's pair geometry runs beside step i+1's network.  With --gpus N > 1 the frames
are sharded in contiguous blocks across N ranks (one process per GPU) and the per-frame feature
records are all-gathered over RCCL each step (weak scaling: B frames per GPU per step).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       (N > 1 is launched by torch.distributed.run; see the driver contract.)
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))

METRIC = "frames/sec end-to-end on TUM 640x480 at 1/2/4/8 MI355X; ATE RMSE vs ref"
H, W = 480, 640
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense fp32 (v_mfma_f32_32x32x2_f32) peak
HBM_PEAK_GBS = 8000.0

# Algorithmic FLOPs of each SuperPoint layer per 640x480 frame (2 * MACs).
LAYER_FLOPS = {
    "conv1_fused": 2 * 480 * 640 * 64 * 1 * 9 + 2 * 480 * 640 * 64 * 64 * 9,  # conv1a + conv1b (+pool)
    "conv2a": 2 * 240 * 320 * 64 * 64 * 9,
    "conv2b_pool": 2 * 240 * 320 * 64 * 64 * 9,
    "conv3a": 2 * 120 * 160 * 128 * 64 * 9,
    "conv3b_pool": 2 * 120 * 160 * 128 * 128 * 9,
    "conv4a": 2 * 60 * 80 * 128 * 128 * 9,
    "conv4b": 2 * 60 * 80 * 128 * 128 * 9,
    "head_a": 2 * 60 * 80 * 512 * 128 * 9,
    "head_b": 2 * 60 * 80 * (65 + 256) * 256,
}


# profiling stage -> kernel symbol (as rocprofv3 reports it) of that stage's dominant launch
STAGE_KERNEL = {
    "conv1_fused": "vs::k_conv3_db<true, 1, true, false>",
    "conv2a": "vs::k_conv_mfma<3, false, 2, false, 16>",
    "conv2b_pool": "vs::k_conv_mfma<3, true, 3, false, 16>",
    "conv3a": "vs::k_conv_mfma<3, false, 4, false, 16>",
    "conv3b_pool": "vs::k_conv_mfma<3, true, 5, false, 16>",
    "conv4a": "vs::k_conv3_db<false, 6, false, true>",
    "conv4b": "vs::k_conv3_db<false, 7, false, true>",
    "head_a": "vs::k_conv3_db<false, 8, false, true>",
    "head_b": "vs::k_conv_mfma<1, false, 9, false, 32>",
}


def pmc_traffic(kernel, batch):
    """HBM bytes per launch of `kernel` from the committed PMC passes (profiles/pmc_traffic.json,
    written by tools/summarize_profiles.py from rocprofv3 FETCH_SIZE / WRITE_SIZE runs of this same
    bench at the same batch), or None when no matching measurement exists."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        doc = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    if doc.get("batch_frames") != batch or kernel not in doc.get("kernels", {}):
        return None, None
    return doc["kernels"][kernel]["hbm_bytes_per_launch"], doc.get("tag")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="frames per GPU per step")
    ap.add_argument("--cpu-frames", type=int, default=12, help="cpu_baseline sample size (processed frames)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--serial", action="store_true", help="wait for each step's geometry before the next network")
    return ap.parse_args()


def cpu_baseline(frames_list, nframes):
    """The CPU restatement (oracle/, test infrastructure) on a bounded sample of the same workload:
    extract + match + F verification + 3D-3D RANSAC (+ the E-matrix fallback when it fails) for
    consecutive frames, OpenMP network."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as oracle
    import vslam_abi
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16, os.cpu_count() or 1))
    with vslam_abi.Context(0) as ctx:
        weights = ctx.weights()
    sample = frames_list[:nframes]
    t0 = time.perf_counter()
    prev = None
    for i, f in enumerate(sample):
        kps, desc = oracle.extract(weights, f["bgr"], nthreads=threads)
        if prev is not None:
            (k1, d1, dep1) = prev
            _, good = oracle.match_ratio(d1, desc)
            _, keep, _, _ = oracle.fmat_verify(k1, kps, good)
            good = good[keep]
            p1 = np.stack([k1["x"][good["query_idx"]], k1["y"][good["query_idx"]]], 1)
            p2 = np.stack([kps["x"][good["train_idx"]], kps["y"][good["train_idx"]]], 1)
            ok3 = oracle.ransac_3d3d(p1, p2, dep1, f["depth"], seed=42 + i)[0]
            if not ok3:  # Slam.cpp:965-984
                ok_e, R_e, t_e = oracle.estimate_motion(p1, p2)[:3]
                if ok_e:
                    oracle.estimate_scale(p1, p2, R_e, t_e, dep1, f["depth"])
        prev = (kps, desc, f["depth"])
    dt = time.perf_counter() - t0
    return {"value": len(sample) / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{len(sample)} consecutive synthetic 640x480 RGB-D frames, oracle/ CPU restatement "
                      f"(OpenMP fp32 SuperPoint, decode/NMS/sample, exact 2-NN match, F-RANSAC "
                      f"verification, 3D-3D RANSAC, E-matrix fallback), "
                      f"{threads} threads, {dt:.1f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import synth
    import vslam_abi
    from vslam_pipeline import DevicePipeline, PoseChain

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    B = args.batch
    n_total = world * B
    # this rank's block of the step's frames + the halo frame before it (cyclic)
    idx = [(rank * B - 1) % n_total] + list(range(rank * B, (rank + 1) * B))
    rendered = synth.frames(sorted(set(idx)), n_total)
    own = [rendered[i] for i in idx[1:]]
    halo = rendered[idx[0]]
    dev = torch.device("cuda", torch.cuda.current_device())
    frames = torch.from_numpy(np.stack([f["bgr"] for f in own])).to(dev)
    depth = torch.from_numpy(np.stack([f["depth"] for f in own])).to(dev)
    depth_prev = torch.from_numpy(halo["depth"]).to(dev)

    ctx = vslam_abi.Context(local if world > 1 else 0)
    pipe = DevicePipeline(ctx, B, H, W, rank=rank, world=world)

    chain = PoseChain()
    n_emat = [0]

    def consume(S):
        # small D2H (one packed pinned copy per step): the host tracker consumes the per-pair motion
        # (3D-3D or the E-matrix fallback, Slam.cpp:961-984)
        ok, R, t, eok, eR, et, esc = pipe.collect(S)
        for p in range(B):
            chain.step(ok[p], R[p], t[p], eok[p], eR[p], et[p], esc[p])
        n_emat[0] += int(eok.sum())
        return int(ok.sum())

    def run_steps(first, count):
        # software pipeline: step i's network is enqueued before the host waits for step i-1's
        # geometry, so the geometry of one step overlaps the network of the next
        n_ok, pending = 0, None
        for i in range(first, first + count):
            S = pipe.submit(frames, depth, frame_count0=i * n_total + rank * B, depth_prev=depth_prev)
            if args.serial:
                n_ok += consume(S)
                continue
            if pending is not None:
                n_ok += consume(pending)
            pending = S
        if pending is not None:
            n_ok += consume(pending)
        return n_ok

    run_steps(0, args.warmup)
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_ok = run_steps(args.warmup, args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    total_frames = world * B * args.steps
    value = total_frames / elapsed

    # dominant kernel: the network layer with the largest device time (HIP events on the stream the
    # kernels run on, accumulated over the timed region)
    conv = {k: v for k, v in prof.items() if k in LAYER_FLOPS}
    dom = max(conv, key=lambda k: conv[k][0])
    dom_ms, dom_launches = conv[dom]
    avg_s = dom_ms / 1e3 / dom_launches
    flops_per_launch = LAYER_FLOPS[dom] * B
    achieved = flops_per_launch / avg_s / 1e12
    net_ms = sum(v[0] for k, v in prof.items() if k in LAYER_FLOPS) / args.steps
    net_flops = sum(LAYER_FLOPS.values()) * B
    stage_ms = {k: round(v[0] / args.steps, 4) for k, v in sorted(prof.items(), key=lambda kv: -kv[1][0])}
    traffic, traffic_tag = pmc_traffic(STAGE_KERNEL.get(dom, ""), B)

    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(own, args.cpu_frames)
        result = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded 640x480 RGB-D room sequence, seeded He-normal SuperPoint weights)",
            "config": {
                "workload": "config[1]: 640x480 RGB-D stream on 1xMI355X - HIP SuperPoint extract + "
                            "ratio-test matching + F-RANSAC verification + 3D-3D RANSAC (E-matrix fallback) "
                            "per processed frame",
                "frames_per_gpu_per_step": B,
                "resolution": "640x480",
                "max_keypoints": 400,
                "ransac_iterations": 200,
                "parallelism": f"frame-sharded x{world}" + (" + RCCL all-gather of features" if world > 1 else ""),
            },
            "roofline": {
                "kernel": f"{STAGE_KERNEL.get(dom, dom)} ({dom})",
                "bound": "mfma",
                "achieved": round(achieved, 3),
                "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": f"profiles/{traffic_tag}_pmc_traffic.json" if traffic_tag else None,
                "avg_launch_ms": round(avg_s * 1e3, 4),
                "flops_per_launch": flops_per_launch,
            },
            "network_tflops": round(net_flops / (net_ms / 1e3) / 1e12, 3),
            "stage_ms_per_step": stage_ms,
            "pairs_ok_3d3d": f"{n_ok}/{world * B * args.steps}" if world == 1 else None,
            "pairs_emat_fallback": f"{n_emat[0]}/{world * B * (args.steps + args.warmup)}" if world == 1 else None,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
