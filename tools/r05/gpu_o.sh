#!/bin/bash
# Round-5: the driver's view — smoke(), then the default bench line (with the CPU baseline)
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || { kill $HB; exit 1; }
timeout -k 10 1000 python -u bench.py > $O/bench.json 2> $O/bench.err || { kill $HB; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], 'roofline', d['roofline']['frac'], d['roofline']['traffic'], 'cpu', json.dumps(d['cpu_baseline'])[:300])
print('fe', d['frontend_batch']['value'], 'mono', d['monocular_hd']['value'], 'ba', json.dumps(d.get('local_ba', {}))[:200])"
kill $HB
