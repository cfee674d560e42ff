#!/bin/bash
# Round-5: CU partition A/B after conv4 F(4x4): more tracker CUs
export TMPDIR=/tmp
O=gpurun_out/r05n4; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
for cfg in "32 8" "40 8" "36 8" "32 8" "40 8"; do
  set -- $cfg
  VS_SLAM_TRACK_CUS=$1 VS_SLAM_SPEC_CUS=$2 VS_SLAM_HOST_PROFILE=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --ba-reps 0 --no-frontend --mono-steps 0 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { kill $HB; tail -5 $O/b_$1_$2.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$1_$2.json').read().strip().splitlines()[-1]); print('track $1 spec $2', d['value'], d['ms_per_step'])"
  grep -E "process_frame|speculation wait|local-map tracking" $O/b_$1_$2.err | tail -3
done
kill $HB
