"""Throughput of the per-frame hot path on MI355X (BASELINE.json metric).

value — end-to-end frames/s of the tracking loop (BASELINE config[1]): every processed 640x480
RGB-D frame goes through
    FeatureExtractor::extract   (SuperPoint fp32 network + decode + greedy NMS + descriptor
                                 sampling, batched B frames per call; FeatureExtractor.cpp:49-259)
    Slam::process_frame         (Slam.cpp:809-1135: ratio matching against the reference keyframe,
                                 F-RANSAC verification, 3D-3D RANSAC with the E-matrix + depth
                                 scale fallback, EKF, local-map tracking, PnP refinement, keyframes
                                 with triangulation / depth points / culling, the visibility sweep,
                                 periodic PnP)
through vs_slam_process_batch_dev (host/tracker.hpp over the HIP kernels), frames resident in HBM
(the PCIe upload a host-buffer caller adds is measured separately: input_upload).  The input is the
non-repeating Pioneer-like drive of synth.pioneer_trajectory (headline_plan: 928 processed frames at
the driver's --steps 20 --warmup 5, timed frames 160-799), the drive tests/test_gpu_headline_drive.py
pins bit for bit against the oracle tracker.  Tracking is sequential within a sequence ("replicas
only"): with --gpus N every rank tracks the SAME drive independently and value is the
frames/s summed over ranks (weak scaling) — a 1 -> N curve of it is linear by construction;
frontend_batch is the frame-batched (sharded, RCCL) scaling figure.  The run ends with the RTS
smoother and the reference's ATE (main.cpp:258-332) against the synthetic ground truth.

frontend_batch — BASELINE config[3], offline batch through the C ABI (vs_batch_submit_dev /
vs_batch_collect, csrc/batch.hip, two steps in flight): each rank extracts its block of B = 318 frames
(the per-GPU shard of the 2,544-image sequence), receives its halo frame's record over the RCCL
point-to-point ring (N > 1), matches the B consecutive pairs ending in its frames and runs F
verification + 3D-3D (+E) per pair.

monocular_hd — BASELINE config[4]: a synthetic 1280x720 stream (the build's HD camera synth.K_HD)
through DepthEstimator::estimate (MiDaS v2.1-small at 256x256, seeded weights: the reference ships
none; its output is kept but, as in the reference, not consumed) and the front end with no depth:
extract + match + F verification + essential-matrix RANSAC / recoverPose per pair, poses chained at
the reference's fallback scale (Slam.cpp:976-980), ATE after sim(3) alignment; MiDaS has its own
roofline line (midas.roofline).

roofline — the dominant throughput-bound kernel (the fused SuperPoint conv1, fp32 MFMA) measured
with HIP events on its stream during the timed region (the tracker extracts each batch in even
chunks of 8 frames on its own stream and CU set, overlapped with tracking; FLOPs per launch =
per-frame FLOPs x frames per launch; traffic per launch = the single-chunk-size PMC pass's bytes per
frame x frames per launch); the latency-bound tracking stages are
reported per frame in stage_ms_per_frame.  cpu_baseline — the oracle (CPU restatement: OpenMP
SuperPoint + the same tracking loop over the CPU stages) on a bounded prefix of the same sequence.

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
# conv1's minimum HBM traffic per frame: the fp32 gray input read once (480 x 640 x 4 B) and the
# pooled 240 x 320 x 64 fp32 output written once
CONV1_MIN_BYTES_PER_FRAME = 480 * 640 * 4 + 240 * 320 * 64 * 4
# post-processing algorithmic bytes per frame: semi read 1,248,000 + 400 x 4 taps x
# 1 KB descriptor gathers 1,638,400 + heatmap write and read 1,228,800 + 420,800 of records out
POST_BYTES_PER_FRAME = 1248000 + 1638400 + 1228800 + 420800
LOOP_FRAMES = 126               # one lap of synth.loop_trajectory (0.3 m/s, 10 processed frames/s)
FRONTEND_STEP_M = 0.01          # config[3]: every image of the 30 Hz stream (FRAME_STEP 1), 0.3 m/s
PIONEER_FRAMES = 848            # freiburg2_pioneer_slam3: 2,544 images, every 3rd processed (README.md:5)
T0 = 1311868164.0               # TUM-like timestamps, 0.1 s per processed frame (FRAME_STEP = 3)

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

# Matrix-core FLOPs the Winograd F(2x2, 3x3) kernels execute per frame (round 3, sp_net.hip k_wino3):
# 16 products per 2 x 2 output tile, input channel and output channel (2.25x fewer than the direct
# conv's 9 per pixel); conv1a (1 -> 64) stays on the vector ALUs inside conv1.  LAYER_FLOPS above stay
# the algorithmic (direct-conv) count the roofline contract asks for.
WINO = os.environ.get("VS_WINO", "1") != "0"
MFMA_FLOPS = dict(LAYER_FLOPS)
if WINO:
    MFMA_FLOPS.update({
        "conv1_fused": 2 * 16 * 240 * 320 * 64 * 64,
        "conv2a": 2 * 16 * 120 * 160 * 64 * 64,
        "conv2b_pool": 2 * 16 * 120 * 160 * 64 * 64,
        "conv3a": 2 * 16 * 60 * 80 * 128 * 64,
        "conv3b_pool": 2 * 16 * 60 * 80 * 128 * 128,
        "conv4a": 2 * 16 * 30 * 40 * 128 * 128,
        "conv4b": 2 * 16 * 30 * 40 * 128 * 128,
        "head_a": 2 * 16 * 30 * 40 * 512 * 128,
    })

# Round 5: the layers with at least VS_WINO4_MIN_WG (default 32) workgroups of 16 x 16 pixels x 64
# output channels per frame run Winograd F(4x4, 3x3) (wino4.hip k_wino4: 36 products per 4 x 4 output
# tile, input and output channel, 2.25 per pixel against F(2x2)'s 4) — every 3x3 layer at 640 x 480,
# conv4a / conv4b (4 x 5 workgroups x 2 channel blocks = 40) included (sp_net.hip:1271-1275); the tiles
# the kernel computes include the padding of its 16 x 16-pixel workgroups (120 x 160: 8 x 10
# workgroups; 60 x 80: 4 x 5).
WINO4 = WINO and os.environ.get("VS_WINO4", "1") != "0"
WINO4_MIN_WG = int(os.environ.get("VS_WINO4_MIN_WG", "32"))
WINO4_LAYERS = ("conv1_fused", "conv2a", "conv2b_pool", "conv3a", "conv3b_pool", "head_a") + (
    ("conv4a", "conv4b") if WINO4_MIN_WG <= 40 else ())
if WINO4:
    MFMA_FLOPS.update({
        "conv1_fused": 2 * 36 * 120 * 160 * 64 * 64,
        "conv2a": 2 * 36 * 60 * 80 * 64 * 64,
        "conv2b_pool": 2 * 36 * 60 * 80 * 64 * 64,
        "conv3a": 2 * 36 * 32 * 40 * 128 * 64,
        "conv3b_pool": 2 * 36 * 32 * 40 * 128 * 128,
        "head_a": 2 * 36 * 16 * 20 * 512 * 128,
    })
    if "conv4a" in WINO4_LAYERS:
        MFMA_FLOPS.update({"conv4a": 2 * 36 * 16 * 20 * 128 * 128, "conv4b": 2 * 36 * 16 * 20 * 128 * 128})

# profiling stage -> symbol prefix (as rocprofv3 reports it) of that stage's dominant kernel; the
# template argument list continues after the prefix (e.g. the chunk width: "<true, 1, true, false, 4>")
STAGE_KERNEL_WINO = {
    "conv1_fused": "vs::k_wino3<true, true",
    "conv2a": "vs::k_wino3<false, false",
    "conv2b_pool": "vs::k_wino3<true, false",
    "conv3a": "vs::k_wino3<false, false",
    "conv3b_pool": "vs::k_wino3<true, false",
    "conv4a": "vs::k_wino3<false, false",
    "conv4b": "vs::k_wino3<false, false",
    "head_a": "vs::k_wino3<false, false",
}
STAGE_KERNEL = {
    "conv1_fused": "vs::k_conv3_db<true, 1, true, false",
    "conv2a": "vs::k_conv_mfma<3, false, 2, false",
    "conv2b_pool": "vs::k_conv_mfma<3, true, 3, false",
    "conv3a": "vs::k_conv_mfma<3, false, 4, false",
    "conv3b_pool": "vs::k_conv_mfma<3, true, 5, false",
    "conv4a": "vs::k_conv3_db<false, 6, false, true",
    "conv4b": "vs::k_conv3_db<false, 7, false, true",
    "head_a": "vs::k_conv3_db<false, 8, false, true",
    "head_b": "vs::k_conv_mfma<1, false, 9, false",
}


STAGE_KERNEL_WINO4 = {
    "conv1_fused": "vs::k_wino4<true, true",
    "conv2a": "vs::k_wino4<false, false",
    "conv2b_pool": "vs::k_wino4<true, false",
    "conv3a": "vs::k_wino4<false, false",
    "conv3b_pool": "vs::k_wino4<true, false",
    "head_a": "vs::k_wino4<false, false",
}
if "conv4a" in WINO4_LAYERS:
    STAGE_KERNEL_WINO4.update({"conv4a": "vs::k_wino4<false, false", "conv4b": "vs::k_wino4<false, false"})

STAGE_KERNEL_DIRECT = dict(STAGE_KERNEL)
if WINO:
    STAGE_KERNEL.update(STAGE_KERNEL_WINO)
if WINO4:
    STAGE_KERNEL.update(STAGE_KERNEL_WINO4)


def kernel_matches(name, prefix):
    """rocprof kernel `name` is the kernel `prefix` names (the prefix ends inside the template list)."""
    return name.startswith(prefix) and name[len(prefix):len(prefix) + 1] in (",", ">")


def pmc_traffic(prefix):
    """HBM bytes per FRAME of the kernel `prefix` names, from the committed PMC passes
    (profiles/pmc_traffic.json, written by tools/summarize_profiles.py from rocprofv3 FETCH_SIZE /
    WRITE_SIZE runs in which every launch of that kernel covered the same number of frames), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        doc = json.load(open(path))
    except (OSError, ValueError):
        return None, None, None
    fpl = doc.get("frames_per_launch")
    for name, k in doc.get("kernels", {}).items():
        if kernel_matches(name, prefix) and fpl:
            return k["hbm_bytes_per_launch"] / fpl, doc.get("tag"), fpl
    return None, None, None


def headline_plan(B, warmup, steps, profile_steps):
    """The headline drive and its step schedule: (n_path, [(k0, k1), ...]) — the processed frames of
    synth.pioneer_trajectory(n_path) and the step ranges run_tracker_steps takes in order: warm-up,
    the timed steps, the extra stage-profiled steps (each range prefetches only inside itself).
    n_path >= the reference sequence's 848 processed frames and >= every frame the schedule tracks."""
    n_path = max(PIONEER_FRAMES, B * (warmup + steps + profile_steps))
    ranges = [(0, warmup), (warmup, warmup + steps)]
    if profile_steps > 0:
        ranges.append((warmup + steps, warmup + steps + profile_steps))
    return n_path, ranges


def run_tracker_steps(slam, bgr, dep, hdep, B, k0, k1):
    """Steps k0..k1-1 of the headline through vs_slam_process_batch_dev: step k = processed frames
    kB..kB+B-1 (device frames bgr[kB], depth dep[kB]; host depth hdep; TUM-like timestamps, FRAME_STEP
    3 ids).  Each batch's extraction is prefetched behind the previous one's (vs_slam_prefetch_batch_dev),
    never across the range's end.  Returns the per-frame process_frame results."""
    out = []
    for k in range(k0, k1):
        if k + 1 < k1:
            i1 = (k + 1) * B
            slam.prefetch_batch_dev(B, bgr[i1].data_ptr(), dep[i1].data_ptr())
        g0 = k * B
        out += list(slam.process_batch_dev(B, bgr[g0].data_ptr(), dep[g0].data_ptr(), hdep[g0:g0 + B],
                                           [T0 + 0.1 * (g0 + j) for j in range(B)], [3 * (g0 + j) for j in range(B)]))
    return out


def launch_plan(gpus, environ, argv):
    """--gpus N: ("run", None) when this process is one rank of an N-rank job (or N == 1);
    ("spawn", cmd) when N > 1 and no launcher started us (WORLD_SIZE unset): the caller starts
    torch.distributed.run with N ranks as a child process, before any GPU call, and relays its
    output and exit code; ("error", msg) when WORLD_SIZE is set and differs from N."""
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return "error", f"--gpus {gpus} but WORLD_SIZE={ws}: the launcher and the flag disagree"
        return "run", None
    if gpus == 1:
        return "run", None
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return "spawn", cmd


def progress(msg):
    """A line on stderr per phase (a profiled run stays visibly alive; stdout keeps the one JSON line)."""
    print(f"[bench] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


def match_roofline(ms_launches, pairs_per_launch, cus, where):
    """The descriptor matcher (k_match, one launch per call) against the fp32 MFMA peak: 2 n^2 256
    FLOP per pair at n = 400 keypoints (every synthetic frame reaches SP_MAX_KEYPOINTS), HIP-event
    time on the stream the kernel runs on.  The peak is scaled to the CUs the launch may use."""
    if not ms_launches or not ms_launches[1] or cus <= 0:
        return None
    ms, launches = ms_launches
    avg_s = ms / 1e3 / launches
    flops = 2.0 * 400 * 400 * 256 * pairs_per_launch
    peak = FP32_MFMA_PEAK_TFLOPS * cus / 256
    ach = flops / avg_s / 1e12
    # csrc/match.hip launch(): one or two pairs per launch take 32 x 32 tiles, more take 64 x 64
    kernel = ("vs::k_match<2, 2, 16, 16, 32, 1, 1, ...> (32 x 32 tiles)" if pairs_per_launch <= 2 else
              "vs::k_match<2, 2, 32, 32, 32, 1, 1, ...> (64 x 64 tiles)")
    return {"where": where, "kernel": kernel, "bound": "mfma",
            "achieved": round(ach, 3), "peak": round(peak, 2), "unit": "TFLOP/s", "frac": round(ach / peak, 4),
            "cus": cus, "pairs_per_launch": pairs_per_launch, "avg_launch_us": round(avg_s * 1e6, 2),
            "us_per_pair": round(avg_s * 1e6 / pairs_per_launch, 2), "launches": launches,
            "flops_per_launch": flops}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5, help="untimed steps (5: the driver's own command)")
    ap.add_argument("--batch", type=int, default=32, help="frames per GPU per step")
    ap.add_argument("--cpu-frames", type=int, default=24, help="cpu_baseline sample size (processed frames)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--frontend-steps", type=int, default=4, help="timed steps of the config[3] batch front end")
    ap.add_argument("--frontend-frames", type=int, default=318,
                    help="config[3] frames per GPU per step (318: the 2,544-image sequence's shard at 8 GPUs)")
    ap.add_argument("--no-frontend", action="store_true")
    ap.add_argument("--ba-reps", type=int, default=5, help="timed calls of the config[2] local-BA window (0: skip)")
    ap.add_argument("--stage-profile", choices=["network", "all", "none"], default="network",
                    help="HIP-event stages inside the timed region (network: the extraction stages only)")
    ap.add_argument("--track-profile-steps", type=int, default=4,
                    help="extra steps after the timed region with every stage profiled (stage_ms_per_frame)")
    ap.add_argument("--mono-steps", type=int, default=4, help="timed steps of the config[4] monocular HD stream")
    ap.add_argument("--render-workers", type=int, default=0,
                    help="processes rendering the synthetic sequence (0: min(16, cpus / ranks); 1 under rocprofv3 "
                         "--pmc, whose preloaded library has initialised the GPU before the fork)")
    return ap.parse_args()


def cpu_baseline(L, nframes, ba=None):
    """The CPU restatement (oracle/, test infrastructure) on the first `nframes` frames of the same
    sequence: OpenMP SuperPoint + decode/NMS/sample, then the same tracking loop (host/tracker.hpp)
    over the CPU stages; and, given the config[2] window `ba`, the CPU local BA on one thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as oracle
    import vslam_abi
    ba_cpu = None
    if ba is not None:
        R, t, P0, kf, pt, uv, iters = ba
        t0 = time.perf_counter()
        o = oracle.local_ba(R, t, P0, kf, pt, uv)
        ms = (time.perf_counter() - t0) * 1e3
        ba_cpu = {"ms_per_call": round(ms, 3), "ms_per_iteration": round(ms / max(int(o[5][0]), 1), 3), "threads": 1,
                  "lm_iterations": int(o[5][0]), "same_lm_trajectory_as_gpu": int(o[5][0]) == iters,
                  "kind": "port", "what": "oracle/orc_ba.cpp (the CPU restatement of Optimizer.cpp:187-599)"}
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16, os.cpu_count() or 1))
    with vslam_abi.Context(0) as ctx:
        weights = ctx.weights()
    S = oracle.Slam()
    t_ext = t_trk = 0.0
    for g in range(nframes):
        t0 = time.perf_counter()
        kps, desc = oracle.extract(weights, L["bgr"][g], nthreads=threads)
        t1 = time.perf_counter()
        S.process(kps, desc, L["depth"][g], T0 + 0.1 * g, 3 * g)
        t_ext += t1 - t0
        t_trk += time.perf_counter() - t1
    dt = t_ext + t_trk
    stages = {k: round(v / nframes * 1e3, 4) for k, v in S.stage_seconds().items()}
    S.close()
    model = "unknown"
    try:
        model = next(ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    table = None
    try:  # config[0] as SURVEY 8(d) defines it: 200 frames at 1, 4 and the box's CPU share (tools/cpu_baseline.py)
        doc = json.load(open(os.path.join(ROOT, "profiles", "cpu_baseline.json")))
        table = {"source": "profiles/cpu_baseline.json (tools/cpu_baseline.py on the GPU box, " + doc.get("tag", "?") + ")",
                 "cpu_model": doc.get("cpu_model"), "frames": doc["runs"][0]["frames"],
                 "runs": [{"threads": r["threads"], "value": r["value"], "unit": r["unit"],
                           "ms_per_frame_extract": r["ms_per_frame"]["extract"],
                           "ms_per_frame_track": r["ms_per_frame"]["track"]} for r in doc["runs"]]}
    except (OSError, ValueError, KeyError, IndexError):
        pass
    return {"value": nframes / dt, "unit": "frames/s", "cores": threads, "kind": "port", "cpu_model": model,
            "config0_table": table,
            "local_ba": ba_cpu,
            "caveats": "a restatement, not the reference binary (OpenCV / ONNX Runtime / g2o are absent): the network "
                       "is the oracle's OpenMP fp32 direct convolution, not ONNX Runtime's MLAS (SURVEY.md 8(d)); "
                       "matching is the exact 2-NN FLANN approximates, AVX2-vectorised and bit-identical to the GPU "
                       "(the reference's randomized kd-tree: ~2-5 ms per 400 x 400 pair, SURVEY.md A7)",
            "ms_per_frame": {"extract": round(t_ext / nframes * 1e3, 3), "track": round(t_trk / nframes * 1e3, 3),
                             **stages},
            "sample": f"first {nframes} frames of the same synthetic 640x480 RGB-D sequence through the oracle/ "
                      f"CPU restatement (OpenMP fp32 SuperPoint + decode/NMS/sample, then Slam::process_frame with "
                      f"exact 2-NN matching, F-RANSAC, 3D-3D RANSAC / E fallback, EKF, local-map tracking, PnP, "
                      f"keyframes), {threads} threads, {dt:.1f} s"}


BA_WINDOW = dict(N=50, M=10000, seed=7, span=3, noise=1.0, pert=0.05)  # SURVEY.md 8(d) BA stress


def ba_bytes_per_iteration(N, M, n_obs):
    """Algorithmic HBM bytes of one local-BA LM iteration: per observation
    the pixel + indices read (24 B) and its 6x3 pose-point block written (144 B); per point its
    position read and written (48 B) and its 3x3 block + gradient (96 B); the 6N x 6N Schur system
    written once and read once by the factorisation (16 B per entry)."""
    return n_obs * (24 + 144) + M * (48 + 96) + (6 * N) ** 2 * 16


def local_ba(ctx, reps):
    """BASELINE config[2]: Optimizer::local_bundle_adjustment (Optimizer.cpp:187-599) on the 50-keyframe
    / 10k-point stress window through vs_local_ba (host arrays in and out, as the reference's call)."""
    import synth
    w = BA_WINDOW
    R, t, P, P0, kf, pt, uv = synth.ba_window(w["N"], w["M"], w["seed"], span=w["span"], noise=w["noise"],
                                              pert=w["pert"])
    g = ctx.local_ba(R, t, P0, kf, pt, uv)  # warm-up: code objects, scratch
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        g = ctx.local_ba(R, t, P0, kf, pt, uv)
    ms = (time.perf_counter() - t0) / reps * 1e3
    prof = ctx.profile_read()
    ctx.profile(False)
    iters = int(g[5][0])
    bpi = ba_bytes_per_iteration(w["N"], w["M"], len(kf))
    res = {"workload": "config[2] local-BA stress window: 50 keyframes / 10k map points / span 3, 1 px noise, 5 cm "
                       "point perturbation (synth.ba_window seed 7), vs_local_ba (Schur complement, blocked "
                       "Cholesky, LM control on the device)",
           "observations": int(len(kf)), "lm_iterations": iters, "accepted_steps": int(g[5][1]),
           "rms_before": round(g[3], 6), "rms_after": round(g[4], 6), "reps": reps,
           "ms_per_call": round(ms, 3), "ms_per_iteration": round(ms / max(iters, 1), 4),
           "roofline": {"bound": "latency (hbm reported)", "algorithmic_bytes_per_iteration": bpi,
                        "achieved": round(bpi / (ms / max(iters, 1) / 1e3) / 1e9, 3), "peak": 8000.0,
                        "unit": "GB/s", "frac": round(bpi / (ms / max(iters, 1) / 1e3) / 8e12, 6)},
           "stage_ms_per_call": {k: round(v[0] / reps, 4) for k, v in prof.items() if v[1]}}
    return res, (R, t, P0, kf, pt, uv, iters)


def batch_schedule(submit, collect, first, count, depth=2):
    """Steps first..first+count-1 through vs_batch_submit_dev / vs_batch_collect with at most `depth`
    steps in flight (the next step's network beside this step's geometry); returns
    the collected motions in step order."""
    out, inflight = [], 0
    for i in range(first, first + count):
        submit(i)
        inflight += 1
        if inflight == depth:
            out.append(collect())
            inflight -= 1
    while inflight:
        out.append(collect())
        inflight -= 1
    return out


def batch_halo_needed(step, rank, world):
    """vs_batch_submit_dev needs the depth of frame rank * B - 1 with a communicator, except on rank 0's
    first step (batch.hip; without one, slot 0 carries over from the previous step)."""
    return world > 1 and (step > 0 or rank > 0)


def share_batch_id(rank, world, make_id, device="cpu", nbytes=128):
    """Rank 0's vs_batch communicator id (make_id() -> bytes) on every rank, broadcast over the torch
    process group (RCCL on the GPU box, gloo in the CPU tests); None for one rank (no communicator)."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    t = torch.zeros(nbytes, dtype=torch.uint8, device=device)
    if rank == 0:
        t.copy_(torch.frombuffer(bytearray(make_id()), dtype=torch.uint8).to(device))
    dist.broadcast(t, 0)
    return bytes(t.cpu().numpy().tobytes())


def frontend_frame_indices(B, rank, world):
    """config[3]'s frames on a rank: its B consecutive frames of the world * B-frame sequence and its halo
    frame (the one before its first; rank 0's is the sequence's last, the previous pass's)."""
    return list(range(rank * B, rank * B + B)), (rank * B - 1) % (world * B)


def frontend_batch(ctx, B, rank, world, steps, warmup, workers=8):
    """BASELINE config[3]: the offline frame-sharded front end through the C ABI (vs_batch_submit_dev /
    vs_batch_collect, csrc/batch.hip — the path INTEGRATION.md gives a C++ driver): per step each rank
    extracts its B frames, receives its halo frame's record over RCCL (point-to-point ring) and runs
    match + F verification + 3D-3D RANSAC + E fallback on the B pairs ending in its frames, the next
    step's network overlapping this step's geometry.  B = the per-GPU shard of the 2,544-image sequence
    (FRAME_STEP 1: 2544 / 8 = 318), so at 8 GPUs one step is the whole sequence.

    Input: world * B distinct frames of the Pioneer-like drive at FRAME_STEP 1 spacing
    (synth.pioneer_trajectory with 0.01 m per frame, a third of the tracked drive's); each rank renders its
    own B frames plus its halo frame (rank * B - 1).  Every step is the same offline pass over the
    sequence, so rank 0's halo after the first step is the sequence's last frame (one seam pair per step)."""
    import torch
    import torch.distributed as dist

    import synth
    import vslam_abi
    n_total = world * B
    dev = torch.device("cuda", torch.cuda.current_device())
    poses = synth.pioneer_trajectory(n_total, step=FRONTEND_STEP_M)
    own, halo_idx = frontend_frame_indices(B, rank, world)
    fb, fd = synth.render_frames(poses, own + [halo_idx], workers=workers)
    frames = torch.from_numpy(fb[:B]).to(dev)
    depth = torch.from_numpy(fd[:B]).to(dev)
    depth_prev = torch.from_numpy(fd[B]).to(dev)
    del fb, fd
    # rank 0's RCCL communicator id, distributed over the torch process group
    uid = share_batch_id(rank, world, vslam_abi.batch_unique_id, dev,
                         getattr(vslam_abi, "VS_BATCH_ID_BYTES", 128))
    bt = vslam_abi.Batch(ctx, B, H, W, rank=rank, world=world, uid=uid)
    s = torch.cuda.current_stream().cuda_stream
    motions = []

    def submit(i):
        halo = depth_prev.data_ptr() if batch_halo_needed(i, rank, world) else None
        bt.submit_dev(frames.data_ptr(), depth.data_ptr(), halo, i * n_total + rank * B, s)

    def run(first, count):
        motions.extend(batch_schedule(submit, bt.collect, first, count))

    run(0, warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    run(warmup, steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    last = motions[-1]
    # the matcher alone on the last step's resident records (B - 1 consecutive pairs of the block per
    # launch, whole chip): inside the pipeline it shares the CUs with the next step's network
    kps_p, desc_p, n_p, nf = bt.features_dev()
    cap = vslam_abi.SP_MAX_KEYPOINTS
    P = nf - 1
    pairs = torch.tensor([[p, p + 1] for p in range(P)], dtype=torch.int32, device=dev)
    raw = torch.zeros(P * cap * vslam_abi.MATCH_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    good = torch.zeros_like(raw)
    nraw = torch.zeros(P, dtype=torch.int32, device=dev)
    ngood = torch.zeros_like(nraw)
    ctx.match_pairs_dev(P, pairs.data_ptr(), nf, desc_p, n_p, cap, 0.75, raw.data_ptr(), nraw.data_ptr(),
                        good.data_ptr(), ngood.data_ptr(), s)
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(20):
        ctx.match_pairs_dev(P, pairs.data_ptr(), nf, desc_p, n_p, cap, 0.75, raw.data_ptr(), nraw.data_ptr(),
                            good.data_ptr(), ngood.data_ptr(), s)
    torch.cuda.synchronize()
    alone = ctx.profile_read().get("match")
    ctx.profile(False)
    # the pipeline's own launches matched B pairs each: the same pair lists (bit-exact kernel)
    assert np.array_equal(ngood.cpu().numpy(), last["n_good"][1:]), "matcher alone differs from the pipeline"
    bt.close()
    # post-processing alone (decode + NMS + top-K + sampling) on 32 frames' network outputs, whole chip:
    # in the pipelines it queues behind the network's workgroups on the same CUs
    nb = min(B, 32)
    hc, wc = H // 8, W // 8
    semi = torch.zeros((nb, hc, wc, vslam_abi.SEMI_CH), dtype=torch.float32, device=dev)
    dgrid = torch.zeros((nb, hc, wc, vslam_abi.DESC_DIM), dtype=torch.float32, device=dev)
    kps = torch.zeros((nb, cap * vslam_abi.KEYPOINT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    desc = torch.zeros((nb, cap, 256), dtype=torch.float32, device=dev)
    n = torch.zeros(nb, dtype=torch.int32, device=dev)
    ctx.network_batch_dev(nb, frames.data_ptr(), H, W, semi.data_ptr(), dgrid.data_ptr(), s)
    ctx.postprocess_batch_dev(nb, semi.data_ptr(), dgrid.data_ptr(), H, W, kps.data_ptr(), desc.data_ptr(),
                              n.data_ptr(), cap, s)
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    reps = 10
    for _ in range(reps):
        ctx.postprocess_batch_dev(nb, semi.data_ptr(), dgrid.data_ptr(), H, W, kps.data_ptr(), desc.data_ptr(),
                                  n.data_ptr(), cap, s)
    torch.cuda.synchronize()
    pp = ctx.profile_read()
    ctx.profile(False)
    post_ms = sum(pp[k][0] for k in ("decode", "nms_rounds", "nms_select", "sample") if k in pp) / (reps * nb)
    post = {"what": "FeatureExtractor.cpp:126-259 after the network (decode, greedy NMS, top-400, border erase, "
                    "descriptor sampling) on 32 frames' resident semi / descriptor grids, alone on the whole chip",
            "frames_per_launch": nb, "ms_per_frame": round(post_ms, 5),
            "stage_ms_per_frame": {k: round(pp[k][0] / (reps * nb), 5) for k in ("decode", "nms_rounds", "nms_select",
                                                                                 "sample") if k in pp},
            "roofline": {"bound": "hbm", "algorithmic_bytes_per_frame": POST_BYTES_PER_FRAME,
                         "achieved": round(POST_BYTES_PER_FRAME / (post_ms / 1e3) / 1e9, 2), "peak": 8000.0,
                         "unit": "GB/s", "frac": round(POST_BYTES_PER_FRAME / (post_ms / 1e3) / 8e12, 5)}}
    del frames, depth
    return {"value": round(world * B * steps / el, 3), "unit": "frames/s", "ms_per_step": round(el / steps * 1e3, 3),
            "_match": alone, "_match_pairs": P, "_match_in_pipeline": prof.get("match"), "steps": steps,
            "frames_per_gpu_per_step": B, "postprocess_alone": post,
            "pairs_3d3d_ok": int(last["ok"].sum()), "pairs_emat_ok": int(last["eok"].sum()),
            "workload": "config[3] offline batch: per-GPU SuperPoint extract + ratio matching + F-RANSAC + 3D-3D "
                        "RANSAC (E fallback) over consecutive frame pairs, no tracking state; the per-GPU shard of "
                        "the 2,544-image sequence (318 frames) per step",
            "path": "C ABI vs_batch_submit_dev / vs_batch_collect (csrc/batch.hip): two steps in flight, the next "
                    "step's network beside this step's geometry",
            "parallelism": f"frame-sharded x{world}" + (" + RCCL point-to-point halo ring over xGMI" if world > 1 else ""),
            "scaling": "weak"}


def monocular_hd(ctx, B, rank, world, steps, warmup, workers):
    """BASELINE config[4] (depth-less): frame-sharded 1280x720 extract + match + F + E per pair."""
    import torch
    import torch.distributed as dist

    import ate
    import synth
    from vslam_pipeline import DevicePipeline, PoseChain
    t_r = time.perf_counter()
    Lh = synth.loop_sequence(LOOP_FRAMES, workers=workers, K=synth.K_HD, w=synth.W_HD, h=synth.H_HD)
    render_s = time.perf_counter() - t_r
    U = LOOP_FRAMES
    n_total = world * B
    dev = torch.device("cuda", torch.cuda.current_device())
    bgr = torch.from_numpy(Lh["bgr"]).to(dev)
    del Lh["bgr"], Lh["depth"]
    import vslam_abi
    midas = vslam_abi.Midas(ctx)  # DepthEstimator (MiDaS v2.1-small, seeded weights) per frame
    pipe = DevicePipeline(ctx, B, synth.H_HD, synth.W_HD, K=synth.K_HD, rank=rank, world=world, monocular=True,
                          midas=midas)
    chain, est, gidx = PoseChain(), [], []

    def run(first, count, track):
        pending = None

        def take(S, i):
            ok, R, t, eok, eR, et, esc = pipe.collect(S)
            if track and world == 1:
                for p in range(B):
                    est.append(chain.step(ok[p], R[p], t[p], eok[p], eR[p], et[p], esc[p])[1])
                    gidx.append((i * n_total + p) % U)
        for i in range(first, first + count):
            idx = torch.tensor([(i * n_total + rank * B + j) % U for j in range(B)], device=dev)
            S = pipe.submit(bgr.index_select(0, idx), None, frame_count0=i * n_total + rank * B)
            if pending is not None:
                take(*pending)
            pending = (S, i)
        if pending is not None:
            take(*pending)

    run(0, warmup, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    run(warmup, steps, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    midas.close()
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    res = {"value": round(world * B * steps / el, 3), "unit": "frames/s", "ms_per_step": round(el / steps * 1e3, 3),
           "steps": steps, "frames_per_gpu_per_step": B, "resolution": "1280x720", "K": list(synth.K_HD),
           "workload": "config[4] monocular stream: per-GPU MiDaS v2.1-small depth (DepthEstimator) + SuperPoint "
                       "extract + ratio matching + F-RANSAC + essential-matrix RANSAC / recoverPose over consecutive "
                       "frame pairs, scale-less (MOTION_SCALE) pose chain; the device-side gather of the batch frames "
                       "is inside the step",
           "parallelism": f"frame-sharded x{world}" + (" + RCCL all-gather of feature records" if world > 1 else ""),
           "render_s": round(render_s, 1)}
    mn = prof.get("midas_net")
    if mn and mn[1]:
        avg_s = mn[0] / 1e3 / mn[1]
        fl = vslam_abi.Midas.flops_per_frame() * B
        res["midas"] = {
            "what": "DepthEstimator::estimate per frame (DepthEstimator.cpp:39-112): MiDaS v2.1-small at 256x256 "
                    "(seeded weights) with the reference's resize / normalisation around it; output kept, not "
                    "consumed (as in the reference)",
            "roofline": {"kernel": "midas_net (all k_mid_conv / k_mid_dw / k_mid_up launches of one batch)",
                         "bound": "mfma", "achieved": round(fl / avg_s / 1e12, 3), "peak": FP32_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(fl / avg_s / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4),
                         "flops_per_frame": vslam_abi.Midas.flops_per_frame(), "frames_per_launch": B,
                         "avg_batch_ms": round(avg_s * 1e3, 3),
                         "note": "shares the chip with the pipeline's SuperPoint network and geometry streams"},
            "stage_ms_per_frame": {k: round(prof[k][0] / (B * steps), 4) for k in ("midas_pre", "midas_net", "midas_post")
                                   if k in prof}}
    if world == 1 and est:
        ts = np.arange(len(est), dtype=np.float64)
        a = ate.compute_ate(ts, np.array(est), ts, Lh["t_wc"][np.array(gidx)])
        res["ate_rmse_m"] = round(a["ate_rmse"], 4)
        res["ate_note"] = "sim(3)-aligned (monocular: scale unobservable), first-pair pose chain per timed window"
    return res


def main():
    args = parse()
    mode, what = launch_plan(args.gpus, os.environ, sys.argv[1:])
    if mode == "error":
        print(f"bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if mode == "spawn":  # no GPU has been touched in this process: the ranks are children
        import subprocess
        progress(f"launching {args.gpus} ranks: {' '.join(what)}")
        sys.exit(subprocess.run(what).returncode)
    import torch
    import torch.distributed as dist

    import ate
    import synth
    import vslam_abi

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    B = args.batch
    dev = torch.device("cuda", torch.cuda.current_device())

    # headline input: the non-repeating Pioneer-like drive of synth.pioneer_trajectory,
    # at least the reference sequence's 848 processed frames (2,544 images at FRAME_STEP 3,
    # main.cpp:1096-1107) and every frame the run tracks distinct; each rank renders every world-th frame
    # and the ranks all-gather them (replicas: every GPU tracks the same drive).  The closed loop
    # (synth.loop_sequence) is the monocular stream's (config[4]); config[3] renders its own drive frames.
    workers = args.render_workers or max(1, min(16, (os.cpu_count() or 1) // max(world, 1)))
    n_path, ranges = headline_plan(B, args.warmup, args.steps,
                                   args.track_profile_steps if args.stage_profile != "all" else 0)
    poses = synth.pioneer_trajectory(n_path)
    mine = list(range(rank, n_path, world))
    pb, pd = synth.render_frames(poses, mine, workers=workers)
    if world > 1:
        per = (n_path + world - 1) // world
        gb = torch.zeros((world, per) + pb.shape[1:], dtype=torch.uint8, device=dev)
        gd = torch.zeros((world, per) + pd.shape[1:], dtype=torch.float32, device=dev)
        lb = torch.zeros((per,) + pb.shape[1:], dtype=torch.uint8, device=dev)
        ld = torch.zeros((per,) + pd.shape[1:], dtype=torch.float32, device=dev)
        lb[:len(mine)].copy_(torch.from_numpy(pb))
        ld[:len(mine)].copy_(torch.from_numpy(pd))
        dist.all_gather_into_tensor(gb, lb)
        dist.all_gather_into_tensor(gd, ld)
        order = [(i % world, i // world) for i in range(n_path)]
        bgr = torch.stack([gb[r, j] for r, j in order])
        dep = torch.stack([gd[r, j] for r, j in order])
        del gb, gd, lb, ld
    else:
        bgr = torch.from_numpy(pb).to(dev)
        dep = torch.from_numpy(pd).to(dev)
    del pb, pd
    Lp = dict(t_wc=np.stack([p[1] for p in poses]), R_wc=np.stack([p[0] for p in poses]))
    hdep_all = dep.cpu().numpy()  # the tracker keeps host copies of live frames' depth
    hdep = [hdep_all[i] for i in range(n_path)]
    Lp["depth"] = hdep_all
    progress(f"{n_path}-frame drive rendered ({len(mine)} frames on this rank)")

    ctx = vslam_abi.Context(local if world > 1 else 0)
    slam = vslam_abi.Slam(ctx, max_batch=B)
    dense = vslam_abi.Dense(ctx)  # main.cpp:1116-1139: every processed frame fused into the dense cloud
    slam.attach_dense(dense)

    progress(f"sequence rendered, tracker ready; {args.warmup} warmup steps")

    def run_steps(k0, k1):
        # never prefetched across the warmup / timed boundary: every timed batch is extracted inside
        # the timed region
        run_tracker_steps(slam, bgr, dep, hdep, B, k0, k1)

    torch.cuda.synchronize()
    run_steps(*ranges[0])
    torch.cuda.synchronize()
    ctx.tie_stats(reset=True)
    # headline: per-stage events on the extraction stages only (the roofline kernel); the tracking
    # stages' per-frame times come from a separate profiled pass (stage_ms_per_frame) so the timed
    # loop carries no event records on the latency-bound tracking stream
    ctx.profile(2 if args.stage_profile == "network" else bool(args.stage_profile == "all"))
    ctx.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(*ranges[1])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    ties = ctx.tie_stats()  # the timed frames' NMS ties (after the timed region: it synchronises)
    progress(f"timed region done: {args.steps} steps in {elapsed:.2f} s")
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    frames_timed = B * args.steps
    value = world * frames_timed / elapsed

    # per-stage times of the tracking stages: a few more steps with every stage's events on (kept
    # out of the timed region; the tracker and the ATE below include these frames)
    prof_trk, frames_trk = prof, frames_timed
    if len(ranges) > 2:
        ctx.profile(True)
        ctx.profile_reset()
        run_steps(*ranges[2])
        torch.cuda.synchronize()
        prof_trk = ctx.profile_read()
        ctx.profile(False)
        frames_trk = B * args.track_profile_steps

    # the PCIe leg a host-buffer caller adds (the reference hands process_frame a host cv::Mat,
    # Frame.cpp:25-29): one batch of BGR + depth from pinned host memory into HBM, timed alone — the
    # headline keeps the frames resident (the boundary takes device pointers)
    upload = None
    if B > 0:
        hb = torch.empty(tuple(bgr[:B].shape), dtype=torch.uint8, pin_memory=True)
        hd = torch.empty(tuple(dep[:B].shape), dtype=torch.float32, pin_memory=True)
        hb.copy_(bgr[:B].cpu())
        hd.copy_(dep[:B].cpu())
        db, dd = torch.empty_like(bgr[:B]), torch.empty_like(dep[:B])
        db.copy_(hb, non_blocking=True)
        dd.copy_(hd, non_blocking=True)
        torch.cuda.synchronize()
        reps = 5
        tu = time.perf_counter()
        for _ in range(reps):
            db.copy_(hb, non_blocking=True)
            dd.copy_(hd, non_blocking=True)
        torch.cuda.synchronize()
        up_s = (time.perf_counter() - tu) / (reps * B)
        nbytes = (hb.numel() + hd.numel() * 4) // B
        upload = {"what": "H2D copy of one batch's BGR + depth (pinned host -> HBM), alone; excluded from value",
                  "bytes_per_frame": int(nbytes), "ms_per_frame": round(up_s * 1e3, 4),
                  "GB_per_s": round(nbytes / up_s / 1e9, 2),
                  "serialised_frames_per_s": round(world / (elapsed / frames_timed + up_s), 3),
                  "note": "serialised = the upload added to every frame's time on its rank with no overlap (an "
                          "upper bound of the cost: a caller can copy the next batch while this one tracks)"}
        del hb, hd, db, dd

    # trajectory quality: RTS smoother, then the reference's ATE against the synthetic ground truth
    slam.finish()
    ids, ts, R, t = slam.trajectory()
    g = np.round((ts - T0) / 0.1).astype(int)
    a = ate.compute_ate(ts, t, ts, Lp["t_wc"][g])
    a_se3 = ate.compute_ate(ts, t, ts, Lp["t_wc"][g], with_scale=False)
    stats = slam.stats_dict()
    dense_points = dense.size()
    ate_t = torch.tensor([a["ate_rmse"]], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ate_t, op=dist.ReduceOp.MAX)

    # dominant throughput-bound kernel: the network layer with the largest device time (HIP
    # events on the stream the kernels run on, accumulated over the timed region)
    # (--stage-profile none, a diagnostic: the network's events come from the extra profiled steps)
    net_prof, net_frames = (prof, frames_timed) if any(k in LAYER_FLOPS for k in prof) else (prof_trk, frames_trk)
    conv = {k: v for k, v in net_prof.items() if k in LAYER_FLOPS}
    dom = max(conv, key=lambda k: conv[k][0]) if conv else "conv1_fused"
    dom_ms, dom_launches = conv.get(dom, (float("nan"), 1))
    # the tracker extracts each batch in even chunks (8, 8, 8, 8 frames at B = 32, tracker.hip
    # enqueue_extraction) overlapped with tracking: a launch covers frames_timed / launches frames
    avg_s = dom_ms / 1e3 / dom_launches
    frames_per_launch = net_frames / dom_launches
    # roofline FLOPs = what the matrix cores execute (Winograd: 2.25x fewer than the direct
    # convolution); the direct-convolution count is reported as the effective rate
    flops_per_launch = MFMA_FLOPS[dom] * frames_per_launch
    achieved = flops_per_launch / avg_s / 1e12
    eff_flops_per_launch = LAYER_FLOPS[dom] * frames_per_launch
    eff_achieved = eff_flops_per_launch / avg_s / 1e12
    net_ms = sum(v[0] for v in conv.values()) if conv else float("nan")
    net_flops = sum(LAYER_FLOPS.values()) * net_frames
    stage_ms = {k: round(v[0] / frames_timed, 4) for k, v in prof.items() if v[1]}
    stage_ms.update({k: round(v[0] / frames_trk, 4) for k, v in prof_trk.items() if v[1] and k not in stage_ms})
    stage_ms = dict(sorted(stage_ms.items(), key=lambda kv: -kv[1]))
    traffic_pf, traffic_tag, traffic_fpl = pmc_traffic(STAGE_KERNEL.get(dom, ""))
    traffic = round(traffic_pf * frames_per_launch) if traffic_pf is not None else None

    # the dominant kernel alone: one extraction chunk (8 frames) and a whole step (B frames) through
    # the network on the whole chip, nothing else running (HIP events on the launch stream)
    alone = {}
    for nb in (8, B):
        semi_t = torch.zeros((nb, 60, 80, vslam_abi.SEMI_CH), dtype=torch.float32, device=dev)
        dg_t = torch.zeros((nb, 60, 80, vslam_abi.DESC_DIM), dtype=torch.float32, device=dev)
        sa = torch.cuda.current_stream().cuda_stream
        ctx.network_batch_dev(nb, bgr[0].data_ptr(), H, W, semi_t.data_ptr(), dg_t.data_ptr(), sa)
        torch.cuda.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        for _ in range(5):
            ctx.network_batch_dev(nb, bgr[0].data_ptr(), H, W, semi_t.data_ptr(), dg_t.data_ptr(), sa)
        torch.cuda.synchronize()
        pa = ctx.profile_read()
        ctx.profile(False)
        ms_l, n_l = pa[dom]
        a_ach = LAYER_FLOPS[dom] * nb / (ms_l / 1e3 / n_l) / 1e12
        net_l = sum(v[0] for k, v in pa.items() if k in LAYER_FLOPS)
        m_ach = MFMA_FLOPS[dom] * nb / (ms_l / 1e3 / n_l) / 1e12
        alone[f"frames_per_launch_{nb}"] = {"avg_launch_ms": round(ms_l / n_l, 4), "achieved": round(m_ach, 3),
                                            "frac": round(m_ach / FP32_MFMA_PEAK_TFLOPS, 4),
                                            "effective_achieved": round(a_ach, 3),
                                            "effective_frac": round(a_ach / FP32_MFMA_PEAK_TFLOPS, 4),
                                            "network_tflops": round(sum(LAYER_FLOPS.values()) * nb * 5 / (net_l / 1e3) / 1e12, 3)}
        del semi_t, dg_t

    track_cus = int(os.environ.get("VS_SLAM_TRACK_CUS", "32"))
    spec_cus = int(os.environ.get("VS_SLAM_SPEC_CUS", "8"))
    if spec_cus <= 0:  # the chain shares the tracking CUs (or, VS_SLAM_SPEC_SET=net, the network's)
        spec_cus = 256 - track_cus if os.environ.get("VS_SLAM_SPEC_SET") == "net" else track_cus
    mroof = {"tracker": match_roofline(prof_trk.get("match"), 1, track_cus,
                                       "tracking loop: one pair per launch on the tracker's "
                                       f"{track_cus}-CU stream (keyframe matches, chains the speculation missed; "
                                       "overlapped with extraction on the rest)"),
             "speculative": match_roofline(prof_trk.get("match_spec"), 1, spec_cus,
                                           "the next frame's speculative chain (frame vs reference keyframe), one pair "
                                           f"per launch on the chain's {spec_cus} CUs, off the critical path")}
    fe = None
    progress("config[3] batch front end")
    if not args.no_frontend and args.frontend_steps > 0:
        fe = frontend_batch(ctx, args.frontend_frames, rank, world, args.frontend_steps, 1, workers)
        P = fe.pop("_match_pairs")
        mroof["frontend_batch"] = match_roofline(fe.pop("_match"), P, 256,
                                                 f"config[3] batch front end's last step: {P} consecutive pairs of the "
                                                 "block per launch on the resident descriptors, alone on the whole "
                                                 f"chip (the pipeline's launches: {args.frontend_frames} pairs)")
        inp = fe.pop("_match_in_pipeline")
        if mroof["frontend_batch"] and inp and inp[1]:
            mroof["frontend_batch"]["in_pipeline_avg_launch_us"] = round(inp[0] * 1e3 / inp[1], 2)

    mono = None
    progress("config[4] monocular HD stream")
    if args.mono_steps > 0:
        mono = monocular_hd(ctx, B, rank, world, args.mono_steps, 1, workers)

    lba, lba_problem = None, None
    if args.ba_reps > 0:
        progress("config[2] local BA stress window")
        lba, lba_problem = local_ba(ctx, args.ba_reps)

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            progress("cpu baseline")
            cpu = cpu_baseline(dict(bgr=bgr[:args.cpu_frames].cpu().numpy(), depth=hdep_all[:args.cpu_frames]),
                               args.cpu_frames, lba_problem)
            if lba is not None and cpu.get("local_ba"):
                lba["cpu_ms_per_call_1thread"] = cpu["local_ba"]["ms_per_call"]
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
            "data": "synthetic (seeded 640x480 RGB-D room rendered along a closed Pioneer-like path, TUM depth "
                    "encoding; seeded He-normal SuperPoint weights: no TUM data or trained weights offline)",
            "config": {
                "workload": "config[1]: 640x480 RGB-D stream, end-to-end Slam::process_frame per processed frame "
                            "(HIP SuperPoint extract + match + F-RANSAC + 3D-3D/E motion + EKF + local-map tracking "
                            "+ PnP + keyframes + loop closure every 200 keyframes, RTS at the end) and the main "
                            "loop's dense voxel fusion of every processed frame (main.cpp:1116-1139), on a "
                            f"non-repeating {n_path}-frame Pioneer-like drive (synth.pioneer_trajectory: the "
                            "reference sequence's 848 processed frames or more; every tracked frame distinct)",
                "path_frames": n_path,
                "timed_frames_distinct": frames_timed,
                "timed_frames": [ranges[1][0] * B, ranges[1][1] * B - 1],
                "parity": "tests/test_gpu_headline_drive.py: this drive and schedule (headline_plan, "
                          "run_tracker_steps) == the oracle tracker bit for bit, and its op log replayed "
                          "through the independent glue restatement (tests/slam_glue_ref.py)",
                "frames_per_gpu_per_step": B,
                "resolution": "640x480",
                "max_keypoints": 400,
                "parallelism": f"replicas x{world} (the same drive on every GPU; tracking is sequential within one: "
                               "a 1 -> N curve of value is linear by construction, frontend_batch is the "
                               "frame-batched scaling figure)",
                "input": "frames resident in HBM before the timed region (device-pointer boundary); the PCIe "
                         "leg of a host-buffer caller: input_upload",
            },
            "ate_rmse_m": round(float(ate_t.item()), 4),
            "ate": {"rank0_rmse_m": round(a["ate_rmse"], 4), "scale": round(a["scale"], 4), "frames": a["n"],
                    "rank0_se3_rmse_m": round(a_se3["ate_rmse"], 4),
                    "reference": "Umeyama sim(3) alignment as main.cpp:258-332 (se3: the same with the scale fixed "
                                 "at 1), synthetic ground truth",
                    "note": "random SuperPoint weights: a median 38 % of the ratio-test matches are geometrically "
                            "correct and the wrong ones are biased toward too-small image motion, so the 3D-3D "
                            "RANSAC accepts consistent wrong motions from the third frame on (DESIGN.md 16.2, "
                            "tools/analyze_bench_trajectory.py); with realistic noise (up to 75 % wrong matches "
                            "without a common motion, 0.7 px, 3 % depth dropouts) the same tracker holds 5-7 mm "
                            "(tests/test_tracker_noisy.py: 58 % wrong over 300 frames, 36 % over 848)"},
            "input_upload": upload,
            "tracker_stats": stats,
            "map_points": stats.get("map_points"), "keyframes": stats.get("keyframes"),
            "nms_ties": dict(ties, note="per timed frame (vs_nms_tie_stats): window / cut ties can change the keypoint "
                                        "set vs the reference's unstable std::sort (FeatureExtractor.cpp:238), order "
                                        "ties only the order of equal-score keypoints in the list; zero = identical "
                                        "for any tie order"),
            "dense_cloud_points": dense_points,
            "roofline": {
                "kernel": f"{STAGE_KERNEL.get(dom, dom)} ({dom})",
                "bound": "mfma",
                "achieved": round(achieved, 3),
                "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per frame, from a PMC "
                                "pass whose launches all covered traffic_pmc_frames_per_launch frames, x frames per "
                                "launch here)",
                "traffic_source": f"profiles/{traffic_tag}_pmc_traffic.json" if traffic_tag else None,
                "traffic_pmc_frames_per_launch": traffic_fpl,
                "algorithmic_bytes_per_launch": round(CONV1_MIN_BYTES_PER_FRAME * frames_per_launch),
                "avg_launch_ms": round(avg_s * 1e3, 4),
                "frames_per_launch": round(frames_per_launch, 3),
                "flops_per_launch": round(flops_per_launch),
                "flops_unit": ("FLOPs the matrix cores execute (Winograd F(4x4, 3x3): 36 products per 4x4 output "
                               "tile, input and output channel); conv1a (1 -> 64, vector ALUs) not counted")
                if WINO4 and dom in WINO4_LAYERS else
                ("FLOPs the matrix cores execute (Winograd F(2x2, 3x3): 16 products per 2x2 output tile, input "
                 "and output channel); conv1a (1 -> 64, vector ALUs) not counted"),
                "algorithm": ("Winograd F(4x4, 3x3), fp32 (wino4.hip k_wino4)" if WINO4 and dom in WINO4_LAYERS else
                              "Winograd F(2x2, 3x3), fp32 (sp_net.hip k_wino3)") if WINO else
                             "direct implicit GEMM, fp32",
                "effective_flops_per_launch": round(eff_flops_per_launch),
                "effective_achieved": round(eff_achieved, 3),
                "effective_frac": round(eff_achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                "effective_note": "direct-convolution FLOPs (the algorithmic work of conv1a + conv1b) / time: the "
                                  "throughput a direct kernel would need to match; with Winograd it can exceed the peak",
                "note": f"network on the extraction stream's CU set (all CUs but the VS_SLAM_TRACK_CUS = {track_cus} "
                        "tracking CUs; " + (f"shared with the VS_SLAM_SPEC_CUS = {spec_cus} CUs of the speculative chains"
                                           if os.environ.get("VS_SLAM_NET_SET", "spec") in ("spec", "all") else
                                           f"without the VS_SLAM_SPEC_CUS = {spec_cus} CUs of the speculative chains") +
                        "), overlapped with tracking; peak is the whole chip's (so frac is a lower bound of the "
                        "utilisation of the CUs the network holds)",
                "alone_whole_chip": alone,
            },
            "match_roofline": mroof,
            "network_tflops": round(net_flops / (net_ms / 1e3) / 1e12, 3),
            "network_tflops_note": "direct-convolution (algorithmic) FLOPs of the whole network / its time; "
                                   "network_mfma_tflops: the FLOPs the matrix cores execute",
            "network_mfma_tflops": round(sum(MFMA_FLOPS.values()) * net_frames / (net_ms / 1e3) / 1e12, 3),
            "stage_ms_per_frame": stage_ms,
            "stage_profile": {"timed_region": args.stage_profile,
                              "network_from": "the timed region" if net_prof is prof else "the extra profiled steps",
                              "tracking_stages_from": (f"{args.track_profile_steps} extra steps after the timed region "
                                                       "with every stage's HIP events on") if prof_trk is not prof
                              else "the timed region"},
            "frontend_batch": fe,
            "monocular_hd": mono,
            "local_ba": lba,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    slam.close()
    ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
