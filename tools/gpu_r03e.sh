#!/bin/bash
# Network-layer A/B (half-height linear tiles for conv4a / conv4b), parity subset, host phase profile.
mkdir -p gpurun_out/r03e
export TMPDIR=/tmp
O=gpurun_out/r03e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tracker_bench.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for mb in 2 1; do
    VS_CONV_LIN_MB=$mb timeout -k 10 120 python -u tools/bench_net.py --tag mb$mb > $O/net_mb${mb}_$r.json 2> $O/net_mb${mb}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/net_mb${mb}_$r.json').read()); print('mb$mb', {k: (v['network_ms_per_launch'], v['layers']['conv4a'], v['layers']['conv4b']) for k, v in d.items() if k.startswith('frames')})"
  done
done
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-frontend \
    --mono-steps 0 --ba-reps 0 > $O/bench_hprof.json 2> $O/bench_hprof.err
rc=$?; echo "hprof rc=$rc"; grep "vs_slam" $O/bench_hprof.err; grep -o '"value": [0-9.]*' $O/bench_hprof.json | head -1
exit $rc
