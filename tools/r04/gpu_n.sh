#!/bin/bash
# PnP RANSAC replay on one wave (prefix-maximum scan, accepted positions walked in order): parity, phases, tracker A/B
export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_pnp.py tests/test_golden.py tests/test_gpu_tracking.py tests/test_gpu_tracker.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker_ideal.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/profile_tracker_phases.py > $O/phases.log 2>&1 || exit 1; python3 -c "import json; d=json.loads(open('$O/phases.log').read().strip().splitlines()[-1]); print(d['pnp_ransac_kcycles_per_call'], d['pnp_hyp_kcycles_per_hypothesis_x100'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --render-workers 1 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); grep -E "k_pnp|k_tlm" $f | cut -d, -f1-4
echo done
