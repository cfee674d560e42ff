#!/bin/bash
# Round-6: speculative next-frame local-map tracking (tracker.hip speculate_next): tracker parity first,
# then the bench A/B (VS_SLAM_SPEC_TLM 1 / 0), the host profile, the out-of-line EPnP stage diff
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06f}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline_drive.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py tests/test_gpu_stationary.py tests/test_gpu_spcf.py tests/test_gpu_dense.py -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -30
[ $rc -eq 0 ] || exit 1
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for v in 1 0 1 0; do
  VS_SLAM_SPEC_TLM=$v timeout -k 10 300 python -u bench.py $H > $O/bench_s$v.json 2> $O/bench_s$v.err || { tail -20 $O/bench_s$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_s$v.json').read().strip().splitlines()[-1])
print('spec_tlm=$v', d['value'], d['ms_per_step'], d['map_points'], d['keyframes'])"
done
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $H > $O/bench_hp.json 2> $O/bench_hp.err || { tail -20 $O/bench_hp.err; exit 1; }
grep "vs_slam" $O/bench_hp.err | head -24
timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py -m gpu -v -s -k "eig_stages" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_eig.log 2>&1
grep -E "stage |PASSED|FAILED" $O/pytest_eig.log | head -20
