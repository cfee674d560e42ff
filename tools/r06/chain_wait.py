#!/usr/bin/env python3
"""Why the tracker waits for the next frame's chain (rocprofv3 --kernel-trace --hip-trace of bench.py).

    python3 tools/r06/chain_wait.py <dir with *_kernel_trace.csv and *_hip_api_trace.csv>

Spec-queue chains (k_match ... the k_copy_bytes after k_emat) are paired with the hipLaunchKernel call that
launched their k_match (thread, time) and with the tracker thread's hipEventSynchronize that returned right
after the chain's copy ended.  Per chain: launch call -> k_match start (queue delay), chain span, and the
wait: when the tracker began waiting relative to the chain's launch and start.  Medians over the chains
the tracker actually waited for (sync returning within 30 us of the copy's end).
"""
import csv
import glob
import os
import statistics as st
import sys


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)[0]
    return list(csv.DictReader(open(f)))


def main(d):
    kern = sorted(load(d, "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    api = load(d, "*hip_api_trace.csv")
    launch_of = {r["Correlation_Id"]: r for r in api if r["Function"].startswith("hipLaunchKernel")}
    # the spec queue: the queue that runs k_match followed by k_fmat
    byq = {}
    for r in kern:
        byq.setdefault(r["Queue_Id"], []).append(r)
    chains = []
    for q, rs in byq.items():
        for i, r in enumerate(rs):
            if "k_match" in r["Kernel_Name"] and i + 4 < len(rs) and "k_fmat" in rs[i + 1]["Kernel_Name"] \
                    and "k_emat" in rs[i + 3]["Kernel_Name"]:
                end = rs[i + 4] if "copy" in rs[i + 4]["Kernel_Name"] else rs[i + 3]
                la = launch_of.get(r["Correlation_Id"])
                chains.append(dict(q=q, start=int(r["Start_Timestamp"]), end=int(end["End_Timestamp"]),
                                   launch=int(la["Start_Timestamp"]) if la else None,
                                   lthread=la["Thread_Id"] if la else None))
    # the tracker thread = the one issuing k_tlm_resolve
    kname = {r["Correlation_Id"]: r["Kernel_Name"] for r in kern}
    tid = next(r["Thread_Id"] for r in api if r["Function"].startswith("hipLaunchKernel")
               and "k_tlm_resolve" in kname.get(r["Correlation_Id"], ""))
    syncs = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api
                    if r["Thread_Id"] == tid and r["Function"] in ("hipEventSynchronize", "hipStreamSynchronize")))
    import bisect
    ends = [s[1] for s in syncs]
    rows = []
    for c in chains:
        j = bisect.bisect_left(ends, c["end"])
        if j < len(syncs) and syncs[j][1] - c["end"] < 30000 and syncs[j][0] < c["end"]:
            ws, we = syncs[j]
            rows.append(dict(qdelay=(c["start"] - c["launch"]) / 1e3 if c["launch"] else float("nan"),
                             span=(c["end"] - c["start"]) / 1e3,
                             wait=(we - ws) / 1e3,
                             wait_after_launch=(ws - c["launch"]) / 1e3 if c["launch"] else float("nan"),
                             wait_after_start=(ws - c["start"]) / 1e3))
    print(f"spec chains: {len(chains)}; waited on by the tracker thread: {len(rows)}")
    if not rows:
        return
    for k in ("qdelay", "span", "wait", "wait_after_launch", "wait_after_start"):
        v = [r[k] for r in rows if r[k] == r[k]]
        print(f"{k:20s} median {st.median(v):8.1f} us   p25 {sorted(v)[len(v) // 4]:8.1f}   p75 {sorted(v)[3 * len(v) // 4]:8.1f}")
    # what the spec queue did between launch and start: kernels of other queues? (the chain waits on an event)
    print("qdelay = hipLaunchKernel(k_match) call -> k_match start; wait_after_launch = the tracker's sync call - that launch")


if __name__ == "__main__":
    main(sys.argv[1])
