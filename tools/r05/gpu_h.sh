#!/bin/bash
# Round-5: matcher largest-first order A/B; vs_batch submit/collect tests; bench line with the config[3] C path
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
for v in 1 0 1 0; do
  VS_MATCH_ORDER=$v timeout -k 10 120 python -u tools/bench_match.py --pairs 32,128,318,512 --reps 10 > $O/m_$v.jsonl 2> $O/m_$v.err || { tail -5 $O/m_$v.err; exit 1; }
  python3 -c "
import json
for l in open('$O/m_$v.jsonl'):
    d = json.loads(l); print('order=$v', d['pairs'], d['us_per_launch'], d['mfma_frac'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; tail -3 $O/pytest.log
timeout -k 10 900 python -u bench.py --no-cpu-baseline --ba-reps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); fe=d['frontend_batch']; m=d['match_roofline']['frontend_batch']
print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'])
print('fe', fe['value'], fe['ms_per_step'], fe['pairs_3d3d_ok'], fe['pairs_emat_ok'], 'match', m['frac'], m['pairs_per_launch'], m['avg_launch_us'], m.get('in_pipeline_avg_launch_us'))
print('mono', d['monocular_hd']['value'])"
echo done
