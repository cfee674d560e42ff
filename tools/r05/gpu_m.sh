#!/bin/bash
# Round-5: full GPU suite + bench line after the overlap fix of vs_batch_submit_dev
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -8; echo "pytest rc=$rc"
if [ $rc -eq 0 ]; then
timeout -k 10 900 python -u bench.py --no-cpu-baseline --ba-reps 0 > $O/bench.json 2> $O/bench.err || { kill $HB; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); fe=d['frontend_batch']; m=d['match_roofline']
print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['map_points'], d['keyframes'])
print('fe', fe['value'], fe['ms_per_step'], 'match fe', m['frontend_batch']['frac'])
print('mono', d['monocular_hd']['value'])"
fi
kill $HB
