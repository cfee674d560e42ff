#!/bin/bash
# Round-6 baseline at HEAD: the driver's own command (--steps 20 --warmup 5) twice, the builder's old
# default (--warmup 2) once, and the host profile of process_frame under both warm-ups
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06a}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
H="--no-cpu-baseline --ba-reps 0 --no-frontend --mono-steps 0"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $H > $O/w5_$r.json 2> $O/w5_$r.err || { tail -20 $O/w5_$r.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 2 $H > $O/w2.json 2> $O/w2.err || { tail -20 $O/w2.err; exit 1; }
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $H > $O/hp_w5.json 2> $O/hp_w5.err || { tail -20 $O/hp_w5.err; exit 1; }
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 2 $H > $O/hp_w2.json 2> $O/hp_w2.err || { tail -20 $O/hp_w2.err; exit 1; }
python3 - <<EOF
import json
for n in ("w5_1", "w5_2", "w2", "hp_w5", "hp_w2"):
    d = json.loads(open("$O/%s.json" % n).read().strip().splitlines()[-1])
    print(n, d["value"], d["ms_per_step"], d["map_points"], d["keyframes"], d["roofline"]["avg_launch_ms"])
EOF
