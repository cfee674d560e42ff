#!/bin/bash
# Second network stream (VS_SLAM_NET_STREAMS=2): tracker parity with it, then a same-box A/B 1 vs 2.
mkdir -p gpurun_out/r03g
export TMPDIR=/tmp
O=gpurun_out/r03g
VS_SLAM_NET_STREAMS=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --track-profile-steps 0"
for r in 1 2 3; do
  for m in 1 2; do
    VS_SLAM_NET_STREAMS=$m timeout -k 10 300 python -u bench.py $ARGS > $O/ns${m}_$r.json 2> $O/ns${m}_$r.err || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$O/ns${m}_$r.json') if l.startswith('{')][-1]); print('ns$m', $r, d['value'], d['roofline']['frac'], d['stage_ms_per_frame'].get('conv1_fused'))"
  done
done
