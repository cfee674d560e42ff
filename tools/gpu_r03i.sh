#!/bin/bash
# Tracker critical path at HEAD: k_pnp_hyp / k_pnp_ransac phase cycles (profiling build), host
# phase profile, and a rocprofv3 kernel trace of the tracker-only bench (per-frame timeline).
mkdir -p gpurun_out/r03i
export TMPDIR=/tmp
O=gpurun_out/r03i
timeout -k 10 600 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py \
    tests/test_gpu_tracker_ideal.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/profile_tracker_phases.py > $O/phases.json 2> $O/phases.err || exit 1
tail -c 1500 $O/phases.json
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-frontend \
    --mono-steps 0 --ba-reps 0 > $O/bench_hostprof.json 2> $O/bench_hostprof.err || exit 1
grep "vs_slam" $O/bench_hostprof.err | head -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 \
    --render-workers 1 > $O/trace.log 2>&1 || exit 1
echo trace ok
