#!/bin/bash
# Round-5: extraction chunk size for the tracker (VS_SLAM_CHUNK 8 = default, 12, 16), headline only
export TMPDIR=/tmp
O=gpurun_out/r05c2; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
for c in 8 16 12 8 16; do
  VS_SLAM_CHUNK=$c timeout -k 10 400 python -u bench.py --no-cpu-baseline --ba-reps 0 --no-frontend --mono-steps 0 > $O/b_$c.json 2> $O/b_$c.err || { tail -5 $O/b_$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$c.json').read().strip().splitlines()[-1])
print('chunk $c', d['value'], d['ms_per_step'], 'conv1 ms/launch', d['roofline'].get('avg_launch_ms'), 'frames/launch', d['roofline'].get('frames_per_launch'))"
done
