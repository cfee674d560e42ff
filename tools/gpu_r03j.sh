#!/bin/bash
# Tracker parity, then a same-box A/B of the headline bench over $VARIANTS (space-separated
# name|env assignments, ',' between assignments), host profile and a kernel trace of the default build.
# r03j: critical-path issue priority (ab/libA.so without, ab/libB.so with); r03k: + early speculative chain.
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracking.py tests/test_gpu_tracker.py tests/test_gpu_tracker_ideal.py tests/test_gpu_stationary.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --track-profile-steps 0"
for r in 1 2 3; do
  for v in $VARIANTS; do
    name=${v%%|*}; envs=${v#*|}; envs=${envs//,/ }
    env $envs timeout -k 10 300 python -u bench.py $ARGS > $O/${name}_$r.json 2> $O/${name}_$r.err || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$O/${name}_$r.json') if l.startswith('{')][-1]); print('$name', $r, d['value'], d['roofline']['frac'])"
  done
done
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/hostprof.json 2> $O/hostprof.err || exit 1
grep "vs_slam" $O/hostprof.err | head -30
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 \
    --render-workers 1 > $O/trace.log 2>&1 || exit 1
echo trace ok
