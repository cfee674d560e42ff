#!/bin/bash
# Tracker parity (bench-scale bit-exact, unit sequences, ideal features, stationary, SPCF replay), then
# the headline bench with the host profile ($TAG output directory).
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py tests/test_gpu_tracker_ideal.py \
    tests/test_gpu_stationary.py tests/test_gpu_spcf.py tests/test_gpu_pnp.py tests/test_gpu_tracking.py -m gpu -x -q \
    --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --track-profile-steps 0"
for r in 1 2; do
  VS_SLAM_HOST_PROFILE=$([ $r = 1 ] && echo 1 || echo 0) timeout -k 10 300 python -u bench.py $ARGS > $O/b$r.json 2> $O/b$r.err || exit 1
  python3 -c "import json; d=json.loads([l for l in open('$O/b$r.json') if l.startswith('{')][-1]); print('run', $r, d['value'])"
done
grep -E "process_frame|extract wait|visibility|phase keyframe|local-map tracking" $O/b1.err | head
