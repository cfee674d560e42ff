#!/bin/bash
# Tracker parity after the local-map call folds its upload / memset into k_tlm_grid, then a
# same-box A/B of the post-processing stream's CU set (VS_SLAM_POST_SET net / track / all).
mkdir -p gpurun_out/r03f
export TMPDIR=/tmp
O=gpurun_out/r03f
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracking.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --track-profile-steps 0"
for r in 1 2 3; do
  for m in net track all; do
    VS_SLAM_POST_SET=$m timeout -k 10 300 python -u bench.py $ARGS > $O/${m}_$r.json 2> $O/${m}_$r.err || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$O/${m}_$r.json') if l.startswith('{')][-1]); print('$m', $r, d['value'], d['roofline']['frac'])"
  done
done
