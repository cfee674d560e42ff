#!/bin/bash
# k_pnp_hyp split into k_pnp_eig (two-wave Jacobi, angles one round ahead) + k_pnp_var: PnP / tracker parity,
# phase cycles, headline A/B vs the committed head (ab/head.so) with the host profile, kernel trace of the chain
export TMPDIR=/tmp
O=gpurun_out/r04y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_pnp.py tests/test_golden.py tests/test_gpu_tracking.py tests/test_gpu_tracker.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker_ideal.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/profile_tracker_phases.py > $O/phases.log 2>&1 || exit 1; python3 -c "import json; d=json.loads(open('$O/phases.log').read().strip().splitlines()[-1]); print(d['pnp_hyp_kcycles_per_hypothesis_x100'])"
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2; do
  for nl in head:ab/head.so new:visual-slam-pipeline_amd/libvslam_hip.so; do
    n=${nl%%:*}; lib=${nl#*:}
    VS_LIB_PATH=$lib VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); print('bench $n $r', d['value'], d['stage_ms_per_frame'].get('solve_pnp'), d['stage_ms_per_frame'].get('track_local_map'))"
    grep -E "process_frame|track_local_map: sync" $O/bench_${n}_$r.err
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --render-workers 1 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); python3 tools/trace_chain.py $f > $O/chain.txt; head -16 $O/chain.txt
rm -f $f
echo done
