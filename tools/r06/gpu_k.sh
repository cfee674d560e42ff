#!/bin/bash
# Round-6: k_fmat at 8 waves, k_ransac3d split over 4 workgroups in the tracker's chain; parity of the
# kernels and the tracker; bench A/B of the split; EPnP out-of-line repro (barrier / own-array variants)
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06k}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 tools/r06/epnp_b_repro > $O/epnp_b_repro.txt 2>&1; tail -5 $O/epnp_b_repro.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_fmat.py tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_headline_drive.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -40
[ $rc -eq 0 ] || exit 1
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for cfg in 4 1 4 1; do
  VS_SLAM_R3_SPLIT=$cfg timeout -k 10 300 python -u bench.py $H > $O/bench_r3_$cfg.json 2> $O/bench_r3_$cfg.err || { tail -20 $O/bench_r3_$cfg.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_r3_$cfg.json').read().strip().splitlines()[-1])
print('r3_split=$cfg', d['value'], d['ms_per_step'], 'conv1', d['roofline']['avg_launch_ms'])"
done
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $H > $O/bench_hp.json 2> $O/bench_hp.err || { tail -20 $O/bench_hp.err; exit 1; }
grep "vs_slam" $O/bench_hp.err | head -24
