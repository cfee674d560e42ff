#!/bin/bash
# Round-6: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) x network streams (1, 2)
export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for cfg in "4 1" "8 1" "8 2" "4 1" "8 1" "8 2"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$1 VS_SLAM_NET_STREAMS=$2 timeout -k 10 300 python -u bench.py $H > $O/b_q$1_s$2.json 2> $O/b_q$1_s$2.err || { tail -20 $O/b_q$1_s$2.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_q$1_s$2.json').read().strip().splitlines()[-1])
print('hwq=$1 streams=$2', d['value'], d['ms_per_step'], 'conv1', d['roofline']['avg_launch_ms'])"
done
