#!/bin/bash
# branch-free Jacobi angles in k_pnp_hyp: parity, phase cycles, kernel time, headline A/B vs committed head (ab/tlm.so)
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_pnp.py tests/test_golden.py tests/test_gpu_tracking.py tests/test_gpu_tracker.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker_ideal.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/profile_tracker_phases.py > $O/phases.log 2>&1 || exit 1; grep -i -A12 "pnp" $O/phases.log | head -30
timeout -k 10 120 python -u tools/profile_ba_phases.py > $O/ba_phases.log 2>&1 || exit 1; tail -2 $O/ba_phases.log
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2; do
  for nl in tlm:ab/tlm.so head:visual-slam-pipeline_amd/libvslam_hip.so; do
    n=${nl%%:*}; lib=${nl#*:}
    VS_LIB_PATH=$lib VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); print('bench $n $r', d['value'], d['stage_ms_per_frame'].get('solve_pnp'), d['stage_ms_per_frame'].get('track_local_map'))"
    grep -E "process_frame|track_local_map: sync" $O/bench_${n}_$r.err
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --render-workers 1 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); grep -E "k_pnp|k_tlm" $f | cut -d, -f1-4
echo done
