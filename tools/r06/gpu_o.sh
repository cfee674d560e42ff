#!/bin/bash
# Round-6: k_tlm_resolve windowed passes (all loads of a round in flight); tracking parity; depth A/B; trace
# bench A/B depth 1 vs 2; host profile; kernel + HIP runtime trace for the chain-wait analysis
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06o}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tracking.py tests/test_gpu_parity.py tests/test_gpu_headline_drive.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -14
[ $rc -eq 0 ] || exit 1
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for d in 2 1; do
  VS_SLAM_SPEC_DEPTH=$d timeout -k 10 300 python -u bench.py $H > $O/bench_d$d.json 2> $O/bench_d$d.err || { tail -20 $O/bench_d$d.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_d$d.json').read().strip().splitlines()[-1])
print('depth=$d', d['value'], d['ms_per_step'])"
done
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $H > $O/bench_hp.json 2> $O/bench_hp.err || { tail -20 $O/bench_hp.err; exit 1; }
grep "vs_slam" $O/bench_hp.err | head -24
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/trace -o trace --output-format csv -- python3 bench.py $H --render-workers 1 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 tools/r06/chain_wait.py $O/trace
python3 tools/trace_chain.py $(ls $O/trace/*kernel_trace.csv $O/trace/*/*kernel_trace.csv 2>/dev/null | head -1) > $O/chain.txt 2>&1; head -40 $O/chain.txt
