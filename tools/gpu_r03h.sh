#!/bin/bash
# HEAD check after the container re-creation: full -m gpu suite, smoke, default bench, kernel stats.
mkdir -p gpurun_out/r03h
export TMPDIR=/tmp
O=gpurun_out/r03h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    -rA > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
tail -c 600 $O/bench_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
echo done
