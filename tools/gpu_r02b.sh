#!/bin/bash
# Round-2 session helper: GPU parity suite, headline bench, tracker host-side profile and the
# k_fmat / k_pnp / k_ransac3d phase counters.  Each GPU step has its own time limit; the chain
# stops at the first abnormal exit (a plain pytest failure, rc 1, still lets the measurements run).
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -q --maxfail=20 -p no:cacheprovider \
    --timeout 200 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > $O/bench.json 2> $O/bench.err &&
echo "bench ok" && tail -c 400 $O/bench.json &&
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-frontend \
    --mono-steps 0 > $O/bench_hprof.json 2> $O/bench_hprof.err && echo "hprof ok" &&
timeout -k 10 200 python -u tools/profile_tracker_phases.py > $O/phases.json 2> $O/phases.err && echo "phases ok"
