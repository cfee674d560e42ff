#!/bin/bash
# Round-5: matcher tile choice for the tracker's one-pair launches (headline only): 32x32 (HEAD) vs 64x64 vs q64t32
export TMPDIR=/tmp
O=gpurun_out/r05m2; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
for t in none default q64t32 none; do
  if [ $t = none ]; then unset VS_MATCH_TILE; else export VS_MATCH_TILE=$t; fi
  VS_SLAM_HOST_PROFILE=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --ba-reps 0 --no-frontend --mono-steps 0 > $O/b_$t.json 2> $O/b_$t.err || { tail -5 $O/b_$t.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]); m=d['match_roofline']
print('tile $t', d['value'], d['ms_per_step'], 'tracker us/pair', m['tracker']['us_per_pair'], 'spec us/pair', m['speculative']['us_per_pair'])"
  grep -E "process_frame|speculation wait" $O/b_$t.err | tail -2
done
