#!/bin/bash
# Round-5: matcher tile variants at large pair counts (config[3] operating points)
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
for t in default k64 k64d k32d w8 w8k64 q64t32 q32t64 default; do
  VS_MATCH_TILE=$t timeout -k 10 120 python -u tools/bench_match.py --pairs 128,318,512,1024 --reps 10 > $O/m_$t.jsonl 2> $O/m_$t.err || { tail -5 $O/m_$t.err; exit 1; }
  python3 -c "
import json
for l in open('$O/m_$t.jsonl'):
    d = json.loads(l); print('$t', d['pairs'], d['us_per_launch'], d['mfma_frac'])"
done
echo done
