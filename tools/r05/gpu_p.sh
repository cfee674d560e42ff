#!/bin/bash
# Round-5: where config[4]'s step goes (kernel totals of the monocular block)
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o mono --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 4 --ba-reps 0 --render-workers 4 > $O/prof.log 2>&1 || { kill $HB; tail -5 $O/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r05p/prof/**/*kernel_stats.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:25]:
    print('%-60s calls %6s total_ms %8.2f avg_us %9.1f %5.1f%%' % (r['Name'][:60], r['Calls'], float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e3, 100*float(r['TotalDurationNs'])/tot))
PY
kill $HB
