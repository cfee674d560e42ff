#!/bin/bash
# Full -m gpu suite, the default bench, then a host-profile bench run (VS_SLAM_HOST_PROFILE=1).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/bench.log | head -1
if [ $rc -ne 0 ]; then exit $rc; fi
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-frontend \
    --mono-steps 0 --ba-reps 0 > gpurun_out/bench_hprof.json 2> gpurun_out/bench_hprof.err
rc=$?; echo "hprof rc=$rc"; grep "vs_slam host" gpurun_out/bench_hprof.err
exit $rc
