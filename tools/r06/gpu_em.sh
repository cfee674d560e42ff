#!/bin/bash
# Round-6 (k_emat split + wave-parallel 5-point): emat parity, the E-using GPU suites, per-call latency
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06em}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_emat.py tests/test_gpu_monocular.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_emat.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $O/pytest_emat.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/r05/bench_emat.py > $O/bench_emat.txt 2>&1 || { tail -5 $O/bench_emat.txt; exit 1; }
cat $O/bench_emat.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o emat --output-format csv -- python3 tools/r05/bench_emat.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs grep -i "emat" | head -5
