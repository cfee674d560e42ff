#!/usr/bin/env python3
"""Per-frame timeline of the tracker's device chain from a rocprofv3 kernel trace of bench.py.

    python3 tools/trace_chain.py gpurun_out/prof_trace/trace_kernel_trace.csv

The tracking queue is the one that runs ``k_tlm_resolve``; a frame's chain starts at ``k_tlm_grid`` (``k_tlm_cand``
since round 6, the grid being built at extraction) and ends at the
first copy after ``k_pnp_ransac`` (the packed result read back: a copy command, or ``k_copy_bytes`` into
coherent host memory).  For the steady-state frames (the median over
all chains) it prints every step's duration and the gap before it, the chain's span, the sum of its kernels, and the
device-idle time from a chain's end to the next chain's start (the host's own part of ``process_frame``).  The
speculative queue (``k_fmat``) is summarised the same way (``k_match`` → ``k_fmat`` → ``k_ransac3d`` → ``k_emat``).
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "")
    return name.split("(")[0].replace("vs::", "")


def chains(rows, first, last):
    """Split one queue's dispatches into chains [first ... last, copy]."""
    out, cur = [], None
    for r in rows:
        k = short(r["Kernel_Name"])
        if k == first:
            cur = [r]
            continue
        if cur is None:
            continue
        cur.append(r)
        if short(cur[-2]["Kernel_Name"]) == last and k in ("__amd_rocclr_copyBuffer", "k_copy_bytes"):
            out.append(cur)
            cur = None
    return out


def summarize(title, ch, rows_by_start):
    pattern = lambda c: tuple(short(r["Kernel_Name"]) for r in c)
    counts = defaultdict(int)
    for c in ch:
        counts[pattern(c)] += 1
    common = max(counts, key=counts.get)
    n_all = len(ch)
    ch = [c for c in ch if pattern(c) == common]  # the steady-state chain (the others: early exits)
    title = f"{title}, {len(ch)} of {n_all} chains with the common kernel sequence"
    steps = defaultdict(list)
    spans, busy, idle = [], [], []
    for c in ch:
        t0 = int(c[0]["Start_Timestamp"])
        prev_end = None
        b = 0
        for i, r in enumerate(c):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            key = f"{i:02d} {short(r['Kernel_Name'])}"
            steps[key].append((e - s, None if prev_end is None else s - prev_end))
            b += e - s
            prev_end = e
        spans.append(prev_end - t0)
        busy.append(b)
    starts = [int(c[0]["Start_Timestamp"]) for c in ch]
    ends = [int(c[-1]["End_Timestamp"]) for c in ch]
    for i in range(len(ch) - 1):
        idle.append(starts[i + 1] - ends[i])
    print(f"## {title}")
    print(f"{'step':32s} {'median us':>10s} {'gap before us':>14s}")
    for key in sorted(steps):
        d = [x[0] for x in steps[key]]
        g = [x[1] for x in steps[key] if x[1] is not None]
        print(f"{key:32s} {statistics.median(d) / 1e3:10.1f} {statistics.median(g) / 1e3 if g else 0:14.2f}")
    print(f"chain span (first start -> last end), median: {statistics.median(spans) / 1e3:.1f} us")
    print(f"sum of the chain's kernels, median:            {statistics.median(busy) / 1e3:.1f} us")
    if idle:
        print(f"queue idle between chains, median:             {statistics.median(idle) / 1e3:.1f} us")
    print()


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    byq = defaultdict(list)
    for r in rows:
        byq[r["Queue_Id"]].append(r)
    for q, rs in byq.items():
        names = {short(r["Kernel_Name"]) for r in rs}
        # round 6: the keypoint grid is built at extraction, so a chain starts at k_tlm_cand
        first = "k_tlm_grid" if "k_tlm_grid" in names and "k_tlm_resolve" in names else "k_tlm_cand"
        if "k_tlm_resolve" in names and first in names:
            summarize(f"tracking queue {q} (local-map tracking + speculative PnP)",
                      [c for c in chains(rs, first, "k_pnp_ransac") if len(c) <= 12], None)
        if "k_fmat<true>" in names:
            summarize(f"speculative queue {q} (match -> F -> 3D-3D -> E)",
                      [c for c in chains(rs, "k_match<2, 2, 16, 16, 32, 1, 1, true, 0>", "k_emat<true>")
                       if len(c) <= 8], None)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_trace/trace_kernel_trace.csv")
