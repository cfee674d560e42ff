"""Per-frame timeline of the tracker's critical-path stream from a rocprofv3 kernel trace CSV:
durations of the local-map / PnP kernels, what overlaps k_pnp_hyp, and the gaps between frames."""
import collections
import csv
import statistics
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"], r["n"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48]
    st = [r for r in rows if "k_pnp_hyp" in r["n"]][0]["Stream_Id"]
    T = sorted([r for r in rows if r["Stream_Id"] == st], key=lambda r: r["s"])
    dur = collections.defaultdict(list)
    for r in T:
        dur[r["n"].split("(")[0]].append((r["e"] - r["s"]) / 1000)
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:40s} n={len(v):5d} median {statistics.median(v):7.1f} us  p90 {sorted(v)[int(0.9 * len(v))]:7.1f}")
    grids = [i for i, r in enumerate(T) if "k_tlm_grid" in r["n"]]
    per = []
    for a, b in zip(grids, grids[1:]):
        per.append((T[b]["s"] - T[a]["s"]) / 1000)
    print("frame period on the stream (k_tlm_grid to k_tlm_grid): median %.1f us" % statistics.median(per))
    crit = []
    for a, b in zip(grids, grids[1:]):
        last = [r for r in T[a:b] if "k_pnp_ransac" in r["n"]]
        if last:
            crit.append((last[-1]["e"] - T[a]["s"]) / 1000)
    print("k_tlm_grid start -> k_pnp_ransac end: median %.1f us" % statistics.median(crit))


if __name__ == "__main__":
    main(sys.argv[1])
