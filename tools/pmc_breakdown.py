"""Per-kernel SQ stall breakdown from tools/pmc_net.sh passes (rocprofv3 counter_collection CSVs):
WAVE_CYCLES split into ACTIVE_INST_ANY / WAIT_INST_ANY / WAIT_ANY, MFMA busy per CU-cycle, LDS
bank-conflict share, and FETCH / WRITE bytes per launch.  Usage: python tools/pmc_breakdown.py DIR"""
import collections
import csv
import glob
import os
import re
import sys


def load(pattern):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.match(r"(?:void )?([\w:]+(?:<[^>]*>)?)", r["Kernel_Name"]).group(1)
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    out = {}
    for k, d in acc.items():
        out[k] = {c: v / n[(k, c)] for c, v in d.items()}
    return out


def main(d):
    for w in ("1", "0"):
        p1 = load(os.path.join(d, f"w{w}p1", "**", "*counter_collection.csv"))
        p2 = load(os.path.join(d, f"w{w}p2", "**", "*counter_collection.csv"))
        print(f"== VS_WINO={w}")
        for k in sorted(p1, key=lambda k: -p1[k].get("SQ_WAVE_CYCLES", 0))[:8]:
            a, b = p1[k], p2.get(k, {})
            wc = a.get("SQ_WAVE_CYCLES", 0) or 1
            gui = a.get("GRBM_GUI_ACTIVE", 0) or 1
            print(f"{k[:46]:46s} active {a.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} wait_inst {a.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}"
                  f" (lds {a.get('SQ_WAIT_INST_LDS', 0) / wc:.2f}) wait_any {a.get('SQ_WAIT_ANY', 0) / wc:.2f}"
                  f" mfma_busy {a.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024 * gui / 8):.2f}"
                  f" lds_conflict {b.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, b.get('SQ_LDS_IDX_ACTIVE', 1)):.2f}"
                  f" valu_insts {b.get('SQ_INSTS_VALU', 0):.3g} lds_insts {b.get('SQ_INSTS_LDS', 0):.3g}")
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        t = load(os.path.join(d, c, "**", "*counter_collection.csv"))
        for k, v in sorted(t.items(), key=lambda kv: -kv[1].get(c, 0))[:6]:
            print(c, k[:46], f"{v.get(c, 0) * 1024 / 1e6:.1f} MB per launch (raw kB x 1024)")


if __name__ == "__main__":
    main(sys.argv[1])
