"""Turn a tools/profile_gpu.sh run (gpurun_out/prof_*) into committed profile artefacts:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc_traffic.json   per-kernel HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE
                                    passes, with the gfx950 correction of MI355X_MICROARCH.md
                                    "HBM": FETCH_SIZE counts half the bytes of a 16-B/lane streaming
                                    read (x2); WRITE_SIZE is exact for 16-B/lane stores.
  profiles/pmc_traffic.json         copy of the latest traffic file (read by bench.py)
  profiles/<tag>_mfma_util.json     per-kernel matrix-core utilisation from the MFMA passes:
                                    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
                                    (GRBM_GUI_ACTIVE is summed over the 8 XCDs; MI355X_MICROARCH.md)
  profiles/<tag>_match_kernel_stats.csv  kernel trace of tools/bench_match.py (1, 32, 512 pairs)

usage: python tools/summarize_profiles.py r03 [frames_per_launch (default 8, the tracker's chunk)]
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", name)
    return m.group(1) if m else name[:80]


def per_kernel(path, counter, grids=None):
    """Mean counter value x 1024 per dispatch of each kernel (FETCH_SIZE / WRITE_SIZE are KB) over
    the dispatches of its most frequent grid size (the tracker's extraction chunk: bench.py's
    network-alone block adds B-frame launches of the same kernels, which must not be averaged in);
    the distinct grid sizes of each kernel's dispatches go to `grids`."""
    per_disp = collections.defaultdict(float)
    names, grid_of = {}, {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d = r.get("Dispatch_Id") or str(len(names))
            per_disp[d] += float(r["Counter_Value"]) * 1024.0
            names[d] = short(r["Kernel_Name"])
            grid_of[d] = r.get("Grid_Size", "")
            if grids is not None and r.get("Grid_Size"):
                grids.setdefault(names[d], set()).add(r["Grid_Size"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, v in per_disp.items():
        agg[names[d]][grid_of[d]].append(v)
    out = {}
    for k, by_grid in agg.items():
        v = max(by_grid.values(), key=len)
        out[k] = sum(v) / len(v)
    return out


def per_dispatch(path):
    """{dispatch: (kernel, grid/wg, {counter: value})} from a --pmc csv (values summed per dispatch)."""
    out = {}
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        k, cs = out.setdefault(d, (short(r["Kernel_Name"]), {}))[:2]
        cs[r["Counter_Name"]] = cs.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def mfma_util(path, label):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, (k, cs) in per_dispatch(path).items():
        for cn, v in cs.items():
            agg[k][cn].append(v)
    res = {}
    for k, cs in agg.items():
        busy = sum(cs["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(cs["SQ_VALU_MFMA_BUSY_CYCLES"])
        gui = sum(cs["GRBM_GUI_ACTIVE"]) / len(cs["GRBM_GUI_ACTIVE"])
        if busy <= 0 or gui <= 0:
            continue
        res[k] = {"source": label, "dispatches": len(cs["GRBM_GUI_ACTIVE"]), "mfma_busy_cycles": busy,
                  "grbm_gui_active": gui, "sq_busy_cycles": sum(cs.get("SQ_BUSY_CYCLES", [0])) / len(cs["GRBM_GUI_ACTIVE"]),
                  "mfma_util": busy / (1024.0 * gui / 8.0)}
    return res


def main():
    tag = sys.argv[1]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(os.path.join(OUT, "prof_trace", "trace_kernel_stats.csv"),
                os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    grids = {}
    fetch = per_kernel(os.path.join(OUT, "prof_fetch", "fetch_counter_collection.csv"), "FETCH_SIZE", grids)
    write = per_kernel(os.path.join(OUT, "prof_write", "write_counter_collection.csv"), "WRITE_SIZE", grids)
    stats = {}
    for r in csv.DictReader(open(os.path.join(OUT, "prof_trace", "trace_kernel_stats.csv"))):
        stats[short(r["Name"])] = float(r["AverageNs"])
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, 0.0)
        w = write.get(k, 0.0)
        kernels[k] = {"fetch_bytes_raw": f, "fetch_bytes_corrected": 2.0 * f, "write_bytes": w,
                      "hbm_bytes_per_launch": 2.0 * f + w, "avg_ns": stats.get(k),
                      "grid_sizes": sorted(grids.get(k, ()))}
    doc = {"tag": tag, "frames_per_launch": batch,
           "note": "FETCH_SIZE x2 (gfx950 16-B/lane streaming-read correction), WRITE_SIZE as is; bytes per launch. "
                   "Taken from bench.py --no-frontend --mono-steps 0: every SuperPoint launch is one tracker "
                   "extraction chunk of frames_per_launch frames (one grid size per network kernel)",
           "kernels": kernels}
    with open(os.path.join(PROF, f"{tag}_pmc_traffic.json"), "w") as fh:
        json.dump(doc, fh, indent=1)
    shutil.copy(os.path.join(PROF, f"{tag}_pmc_traffic.json"), os.path.join(PROF, "pmc_traffic.json"))
    util = {}
    for sub, name, label in (("prof_mfma", "mfma", "bench.py"), ("prof_match_mfma", "match_mfma", "tools/bench_match.py")):
        path = os.path.join(OUT, sub, f"{name}_counter_collection.csv")
        if os.path.exists(path):
            util.update(mfma_util(path, label))
    if util:
        with open(os.path.join(PROF, f"{tag}_mfma_util.json"), "w") as fh:
            json.dump({"tag": tag, "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)",
                       "kernels": util}, fh, indent=1)
        for k, v in sorted(util.items(), key=lambda kv: -kv[1]["mfma_busy_cycles"])[:8]:
            print(f"{k:40s} mfma util {v['mfma_util']:.3f} ({v['source']})")
    mt = os.path.join(OUT, "prof_match", "match_kernel_stats.csv")
    if os.path.exists(mt):
        shutil.copy(mt, os.path.join(PROF, f"{tag}_match_kernel_stats.csv"))
    top = sorted(kernels.items(), key=lambda kv: -(kv[1]["avg_ns"] or 0))[:8]
    for k, v in top:
        print(f"{k:40s} avg {v['avg_ns'] or 0:12.0f} ns  hbm {v['hbm_bytes_per_launch'] / 1e9:8.3f} GB")


if __name__ == "__main__":
    main()
