#!/bin/bash
# Round-4 opening check: headline bench (default arguments) + host profile of process_frame.
export TMPDIR=/tmp
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 > $O/bench_hostprof.json 2> $O/bench_hostprof.err || exit 1
echo done
