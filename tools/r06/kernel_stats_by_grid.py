#!/usr/bin/env python3
"""rocprofv3 kernel statistics split by launch grid (conv1's 8-frame launches apart from
the other batch sizes), from a --kernel-trace CSV.

    python3 tools/r06/kernel_stats_by_grid.py <kernel_trace.csv or dir> [--by-queue] [name substring ...] > stats.csv

One row per (kernel, grid x/y/z, workgroup x[, queue]): calls, total / average / min / max duration in ms.
With name substrings, only kernels whose name contains one of them.  --by-queue also splits by HSA queue
(bench.py's in-pipeline network runs on the extraction stream's queue, its network-alone block on another).
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(path, names, by_queue=False):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if names and not any(n in k for n in names):
            continue
        key = (k, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"]) + \
            ((r["Queue_Id"],) if by_queue else ())
        acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    w = csv.writer(sys.stdout)
    w.writerow(["Kernel_Name", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Workgroup_Size_X"] +
               (["Queue_Id"] if by_queue else []) + ["Calls", "TotalDurationMs", "AverageMs", "MinMs", "MaxMs"])
    for key, d in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        w.writerow(list(key) + [len(d), f"{sum(d):.4f}", f"{sum(d) / len(d):.4f}", f"{min(d):.4f}", f"{max(d):.4f}"])


if __name__ == "__main__":
    args = sys.argv[2:]
    main(sys.argv[1], [a for a in args if a != "--by-queue"], "--by-queue" in args)
