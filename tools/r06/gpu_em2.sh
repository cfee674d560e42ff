#!/bin/bash
# Round-6 k_emat over the whole budget (bound-skipping workgroups, wave-scan replay): E parity and the
# suites that run E (monocular, config[3] batch vs oracle, the headline drive), per-call latency, the bench line
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06em2}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_emat.py tests/test_gpu_monocular.py tests/test_gpu_batch.py tests/test_gpu_headline_drive.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $O/pytest.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/r05/bench_emat.py > $O/bench_emat.txt 2>&1 || { tail -5 $O/bench_emat.txt; exit 1; }
cat $O/bench_emat.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'fe', d['frontend_batch']['value'], 'mono', d['monocular_hd']['value'], d['monocular_hd'].get('ms_per_step'), 'ba', d['local_ba']['ms_per_call'], 'emat/frame', d['stage_ms_per_frame'].get('emat_motion'))"
