#!/bin/bash
# (the NTB variants were removed after this sweep: profiles/r04m_match_train_loop_sweep.txt)
# Matcher: NTB train blocks per workgroup (top-2 kept in registers, one publish per query block):
# bit-exactness of every variant (match parity tests), then event-timed launches at P = 1, 32, 128
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
for t in q32t32 q32tb2 q32tb4 default tb2 tb4 tb7; do
  VS_MATCH_TILE=$t timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "match" -p no:cacheprovider > $O/parity_$t.log 2>&1 || { echo "parity $t FAILED"; tail -20 $O/parity_$t.log; exit 1; }
  echo "parity $t $(tail -1 $O/parity_$t.log)"
done
for r in 1 2; do
  for t in q32t32 q32tb2 q32tb4 default tb2 tb4 tb7; do
    VS_MATCH_TILE=$t timeout -k 10 120 python tools/bench_match.py --pairs 1,32,128 --reps 30 > $O/bench_${t}_$r.jsonl 2> $O/bench_${t}_$r.err || { echo "bench $t FAILED"; tail -5 $O/bench_${t}_$r.err; exit 1; }
    python3 -c "
import json
for l in open('$O/bench_${t}_$r.jsonl'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print('$t', $r, d['pairs'], d['us_per_launch'], d['mfma_frac'])"
  done
done
echo done
