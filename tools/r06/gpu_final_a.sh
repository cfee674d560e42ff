#!/bin/bash
# Round-6 final (A): the whole GPU suite as the driver runs it, smoke(), the default bench line
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06z}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $O/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
tail -3 $O/smoke.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'fe', d['frontend_batch']['value'], 'mono', d['monocular_hd']['value'], 'ba', d['local_ba']['ms_per_call'], 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
