#!/usr/bin/env python3
"""Where the tracker thread's time goes per frame, from a rocprofv3 --hip-trace (+ --kernel-trace) of bench.py.

    python3 tools/r06/host_timeline.py <dir with *_hip_api_trace.csv and *_kernel_trace.csv>

Frames are delimited on the thread that issues k_tlm_resolve launches (the tracker's own thread): one frame = from
one k_tlm_resolve launch call to the next.  Per frame it sums the HIP API time of that thread by function and
reports the rest as host compute (the tracker's own C++: EKF, bookkeeping, parsing), medians over the
steady-state frames; then the device chain of the same frames (first tracking kernel start -> the copy after
k_pnp_ransac) for comparison.
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def load(pattern):
    fs = glob.glob(pattern, recursive=True)
    if not fs:
        sys.exit(f"no file matches {pattern}")
    with open(fs[0]) as f:
        return list(csv.DictReader(f))


def main(d):
    api = load(os.path.join(d, "**", "*hip_api_trace.csv"))
    kern = load(os.path.join(d, "**", "*kernel_trace.csv"))
    # correlation id -> kernel name, so the launch call of k_tlm_grid can be found
    kname = {r["Correlation_Id"]: r["Kernel_Name"] for r in kern}
    launches = [r for r in api if r["Function"].startswith("hipLaunchKernel") or r["Function"] == "hipExtLaunchKernel"]
    tid = None
    for r in launches:
        if "k_tlm_resolve" in kname.get(r["Correlation_Id"], ""):
            tid = r["Thread_Id"]
            break
    if tid is None:
        sys.exit("no k_tlm_resolve launch found")
    mine = sorted((r for r in api if r["Thread_Id"] == tid), key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in mine
             if r["Function"].startswith("hipLaunchKernel") and "k_tlm_resolve" in kname.get(r["Correlation_Id"], "")]
    per = []
    for a, b in zip(marks, marks[1:]):
        fn = defaultdict(float)
        cnt = defaultdict(int)
        busy = 0.0
        for r in mine:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s < a or s >= b:
                continue
            fn[r["Function"]] += (e - s) / 1e3
            cnt[r["Function"]] += 1
            busy += (e - s) / 1e3
        per.append(((b - a) / 1e3, busy, fn, cnt))
    per = per[len(per) // 8:]  # steady state
    wall = statistics.median(p[0] for p in per)
    busy = statistics.median(p[1] for p in per)
    print(f"frames: {len(per)}   tracker thread {tid}")
    print(f"frame period (k_tlm_resolve launch to launch), median: {wall:8.1f} us")
    print(f"  HIP API time on the thread, median:            {busy:8.1f} us")
    print(f"  host compute (the rest), median:               {wall - busy:8.1f} us")
    names = sorted({k for p in per for k in p[2]}, key=lambda k: -statistics.mean(p[2].get(k, 0.0) for p in per))
    print(f"{'function':40s} {'mean us/frame':>14s} {'calls/frame':>12s} {'us/call':>9s}")
    for k in names[:25]:
        m = statistics.mean(p[2].get(k, 0.0) for p in per)
        c = statistics.mean(p[3].get(k, 0) for p in per)
        print(f"{k:40s} {m:14.1f} {c:12.2f} {m / max(c, 1e-9):9.2f}")
    # other threads (helpers: the async enqueue of the next batch, the speculative chain launcher)
    others = defaultdict(float)
    for r in api:
        if r["Thread_Id"] != tid:
            others[r["Thread_Id"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    span = (marks[-1] - marks[0]) / 1e3 if len(marks) > 1 else 1.0
    for t, v in sorted(others.items(), key=lambda kv: -kv[1])[:4]:
        print(f"thread {t}: HIP API busy {100 * v / span:5.1f} % of the traced frames' span")


if __name__ == "__main__":
    main(sys.argv[1])
