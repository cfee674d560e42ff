"""The config[0] CPU baseline as planned: the CPU restatement
(oracle/, test infrastructure: OpenMP fp32 SuperPoint + decode/NMS/sample, then the tracking loop
host/tracker.hpp over the CPU stages) on N processed frames of the bench's synthetic 640x480
RGB-D sequence, at several thread counts, with the CPU model and a per-stage split.

Only SuperPoint is multi-threaded (the reference's tracking loop is sequential), so "threads" is
the OpenMP width of the extraction.  Weights: the product's seeded He-normal weights restated in
numpy (tools/oracle_long_run.py), so the run needs no GPU.

Usage: python tools/cpu_baseline.py [--frames 200] [--threads 1,4,16] [--out profiles/r02_cpu_baseline.json]
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "visual-slam-pipeline_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

LOOP = 126
T0 = 1311868164.0


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def run(weights, L, frames, nt):
    import oracle_py as oracle
    S = oracle.Slam()
    t_ext = t_trk = 0.0
    for g in range(frames):
        t0 = time.perf_counter()
        kps, desc = oracle.extract(weights, L["bgr"][g % LOOP], nthreads=nt)
        t1 = time.perf_counter()
        S.process(kps, desc, L["depth"][g % LOOP], T0 + 0.1 * g, 3 * g)
        t2 = time.perf_counter()
        t_ext += t1 - t0
        t_trk += t2 - t1
        if (g + 1) % 10 == 0:
            print(f"  threads={nt} frame {g + 1}/{frames}: {(g + 1) / (t_ext + t_trk):.3f} frames/s", flush=True)
    st = S.stage_seconds()
    S.close()
    total = t_ext + t_trk
    return {"threads": nt, "frames": frames, "value": round(frames / total, 4), "unit": "frames/s",
            "seconds": round(total, 2),
            "ms_per_frame": {"extract": round(t_ext / frames * 1e3, 3), "track": round(t_trk / frames * 1e3, 3),
                             **{k: round(v / frames * 1e3, 4) for k, v in st.items()}}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--threads", default=None, help="comma list (default 1,4,<OMP_NUM_THREADS or nproc>)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--tag", default=None, help="round tag recorded in the output (e.g. r04)")
    args = ap.parse_args()
    import synth
    from oracle_long_run import _weights
    nmax = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    threads = [int(x) for x in args.threads.split(",")] if args.threads else sorted({1, 4, nmax})
    L = synth.loop_sequence(LOOP, workers=min(8, os.cpu_count() or 1))
    w = _weights()
    res = {"what": "config[0] CPU baseline: oracle/ CPU restatement (OpenMP fp32 SuperPoint extract, then "
                   "Slam::process_frame over the CPU stages), bench.py's synthetic 640x480 RGB-D closed loop",
           "cpu_model": cpu_model(), "nproc": os.cpu_count(), "tag": args.tag,
           "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
           "runs": []}
    for nt in threads:
        r = run(w, L, args.frames, nt)
        res["runs"].append(r)
        print(json.dumps(r), flush=True)
    print(json.dumps({k: v for k, v in res.items() if k != "runs"}), flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
