#!/bin/bash
# Round-5: EPnP eigen stage rewrite (QR null space + tridiagonal multisection / inverse iteration):
# PnP + tracker parity, k_pnp_hyp phase cycles, tracker bench, full bench line
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pnp.py tests/test_golden.py tests/test_gpu_tracker_ideal.py tests/test_gpu_tracker_bench.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/profile_tracker_phases.py > $O/phases.json 2> $O/phases.err || { tail -5 $O/phases.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/phases.json').read().strip().splitlines()[-1]); print('pnp phases', d.get('pnp_hyp_kcycles_per_hypothesis_x100'))"
timeout -k 10 900 python -u bench.py --no-cpu-baseline --ba-reps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); fe=d['frontend_batch']; m=d['match_roofline']['frontend_batch']
print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'], d.get('map_points'), d.get('keyframes'))
print('fe', fe['value'], fe['ms_per_step'], fe['pairs_3d3d_ok'], fe['pairs_emat_ok'], 'match', m['frac'], m['pairs_per_launch'], m['avg_launch_us'], m.get('in_pipeline_avg_launch_us'))
print('tracker', json.dumps(d.get('tracker_kernels', d.get('tracker', {})))[:600])
print('mono', d['monocular_hd']['value'])"
echo done
