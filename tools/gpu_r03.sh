#!/bin/bash
# Round-3 GPU session: the -m gpu suite, the default bench, then (PROFILE=1) the rocprofv3 passes of
# tools/profile_gpu.sh.  Every GPU step has its own time limit; the chain stops at the first
# abnormal exit (fault / abort / timeout).  Output under gpurun_out/.
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -n "$PROFILE" ]; then
  bash tools/profile_gpu.sh; rc=$?; echo "profile rc=$rc"; exit $rc
fi
