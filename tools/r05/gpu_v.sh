#!/bin/bash
# Round-5: the full GPU suite and the default bench line after the post-processing fusion
export TMPDIR=/tmp
O=gpurun_out/${GPU_V_OUT:-r05v}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], 'roofline', d['roofline']['frac'], d['roofline']['traffic'], 'cpu', json.dumps(d['cpu_baseline'])[:200])
print('fe', d['frontend_batch']['value'], 'post', json.dumps(d['frontend_batch'].get('postprocess_alone'))[:300], 'mono', d['monocular_hd']['value'])
print('stages', d['stage_ms_per_frame'])"
