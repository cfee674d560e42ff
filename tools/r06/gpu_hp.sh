#!/bin/bash
# Round-6 HEAD: host profile of the headline (where the tracker thread waits) and a kernel + HIP trace for the chain table
export TMPDIR=/tmp
O=gpurun_out/r06hp; mkdir -p $O
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $H > $O/bench_hp.json 2> $O/bench_hp.err || { tail -20 $O/bench_hp.err; exit 1; }
grep "vs_slam" $O/bench_hp.err | head -24
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/trace -o trace --output-format csv -- python3 bench.py $H --render-workers 1 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 tools/r06/chain_wait.py $O/trace
python3 tools/trace_chain.py $(ls $O/trace/*kernel_trace.csv $O/trace/*/*kernel_trace.csv 2>/dev/null | head -1) > $O/chain.txt 2>&1; head -40 $O/chain.txt
