"""Summarise tools/bench_net.py JSON lines in a directory: network ms per launch and per-layer ms /
fraction of the fp32 MFMA peak (direct-conv FLOPs) for every net_*.json."""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "net_*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    for k, v in d.items():
        if not k.startswith("frames"):
            continue
        lay = " ".join(f"{n}={x['ms_per_launch']:.3f}" for n, x in v["layers"].items() if "conv" in n or "head" in n)
        print(os.path.basename(f), k, f"net={v['network_ms_per_launch']:.3f}", lay)
