#!/bin/bash
# Noisy-feature tracker test on the GPU, the config[0] CPU table (200 frames at 1/4/16 threads), bench.
export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tracker_noisy.py -m gpu -x -v -s --timeout 500 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
OMP_NUM_THREADS=16 timeout -k 10 900 python -u tools/cpu_baseline.py --frames 200 --threads 1,4,16 --tag r04 --out $O/cpu_baseline.json > $O/cpu_baseline.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo done
