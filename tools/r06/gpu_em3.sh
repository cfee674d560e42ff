#!/bin/bash
# Round-6: k_emat split A/B on config[4] (monocular HD: E on all 32 pairs per step beside the network) and a
# kernel trace of the per-call latency tool (k_emat launch durations)
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06em3}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
H="--no-cpu-baseline --no-frontend --steps 1 --warmup 1 --ba-reps 0 --mono-steps 8"
for sp in 125 8 16 125 8 16; do
  VS_EMAT_SPLIT=$sp timeout -k 10 300 python -u bench.py $H > $O/m_$sp.json 2> $O/m_$sp.err || { tail -20 $O/m_$sp.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/m_$sp.json').read().strip().splitlines()[-1]); m=d['monocular_hd']
print('split=$sp mono', m['value'], m.get('ms_per_step'), json.dumps({k: v for k, v in m.items() if 'emat' in k or 'stage' in k})[:300])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o emat --output-format csv -- python3 tools/r05/bench_emat.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 tools/r06/kernel_stats_by_grid.py $O/prof k_emat > $O/emat_by_grid.csv; cat $O/emat_by_grid.csv
