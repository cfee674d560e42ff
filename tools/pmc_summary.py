"""Sum rocprofv3 PMC counters per kernel dispatch from a rocpd SQLite database (rocprofv3 --pmc
without --output-format csv) and print per-kernel averages.

    python tools/pmc_summary.py gpurun_out/<dir>/<name>_results.db [kernel-substring]"""
import collections
import sqlite3
import sys


def main():
    db, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, sum(value), max(duration), grid_size, "
                     "workgroup_size, lds_block_size, vgpr_count, accum_vgpr_count from counters_collection "
                     "group by dispatch_id, counter_name").fetchall()
    per = collections.defaultdict(dict)
    meta = {}
    for d, k, cn, v, dur, gs, ws, lds, vg, ag in rows:
        if pat and pat not in k:
            continue
        per[d][cn] = v
        meta[d] = (k, dur, gs, ws, lds, vg, ag)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, cs in per.items():
        k, dur, gs, ws, lds, vg, ag = meta[d]
        key = (k[:90], gs // ws)
        agg[key]["duration_ns"].append(dur)
        for cn, v in cs.items():
            agg[key][cn].append(v)
    for (k, nwg), cs in agg.items():
        print(f"{k}  workgroups={nwg}  dispatches={len(cs['duration_ns'])}")
        for cn, vs in sorted(cs.items()):
            print(f"    {cn:28s} {sum(vs) / len(vs):16.1f}")


if __name__ == "__main__":
    main()
