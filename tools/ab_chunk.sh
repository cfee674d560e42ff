#!/bin/bash
# Same-box A/B of the extraction chunk size (VS_SLAM_CHUNK) on the headline bench (tracker only).
mkdir -p gpurun_out/ab_chunk
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for round in 1 2; do
  for c in ${CHUNKS:-8 16 11}; do
    VS_SLAM_CHUNK=$c timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_chunk/c${c}_r${round}.json 2> gpurun_out/ab_chunk/c${c}_r${round}.err || exit 1
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_chunk/c${c}_r${round}.json') if l.startswith('{')][-1]); print('chunk ${c} round ${round}', d['value'], d['roofline']['frac'], d['roofline']['frames_per_launch'])"
  done
done
