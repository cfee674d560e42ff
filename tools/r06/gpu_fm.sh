#!/bin/bash
# Round-6: k_fmat's first chunk split over 8 workgroups: F parity (incl. forced splits), the suites that run F
# (config[3] batch vs oracle, tracker, headline drive), the phase profile, headline A/B vs the previous library
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06fm}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_fmat.py tests/test_gpu_batch.py tests/test_gpu_tracker.py tests/test_gpu_headline_drive.py tests/test_gpu_tracker_bench.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $O/pytest.log | tail -5
[ $rc -eq 0 ] || exit 1
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for t in new old new old new old; do
  L=""; [ $t = old ] && L=$PWD/tools/r06/oldlib/libvslam_hip.so
  VS_LIB_PATH=$L timeout -k 10 300 python -u bench.py $H > $O/b_$t.json 2> $O/b_$t.err || { tail -20 $O/b_$t.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']
print('$t', d['value'], d['ms_per_step'], 'fmat', s.get('fmat_ransac'), 'match_spec', s.get('match_spec'), 'r3d', s.get('ransac3d'), 'conv1', s.get('conv1_fused'))"
done
