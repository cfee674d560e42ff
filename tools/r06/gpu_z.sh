#!/bin/bash
# Round-6: which HSA queues the tracker's streams land on with two network streams (kernel trace), at the
# default hardware-queue count and at GPU_MAX_HW_QUEUES=8
export TMPDIR=/tmp
O=gpurun_out/r06zq; mkdir -p $O
H="--steps 2 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --render-workers 1 --track-profile-steps 0"
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q VS_SLAM_NET_STREAMS=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/q$q -o q --output-format csv -- python3 bench.py $H > $O/q$q.log 2>&1 || { tail -5 $O/q$q.log; exit 1; }
  python3 - <<PY
import csv, glob, collections
f = glob.glob("$O/q$q/**/*kernel_trace.csv", recursive=True)[0]
by = collections.defaultdict(collections.Counter)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    k = "net" if "k_wino4" in n or "k_conv_mfma" in n or "k_gray" in n else "tlm" if "k_tlm" in n or "k_pnp" in n else "chain" if "k_fmat" in n or "k_ransac3d" in n else "post" if "k_nms" in n or "k_sample" in n else "other"
    by[r["Queue_Id"]][k] += 1
print("GPU_MAX_HW_QUEUES=$q", {q: dict(c) for q, c in by.items()})
PY
done
