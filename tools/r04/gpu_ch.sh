#!/bin/bash
# extraction chunk size A/B at HEAD (VS_SLAM_CHUNK 8 / 16 / 4 / 11): headline bench with the host profile, two rounds
export TMPDIR=/tmp
O=gpurun_out/r04ch; mkdir -p $O
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2; do
  for c in 8 16 4 11; do
    VS_SLAM_CHUNK=$c VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_c${c}_$r.json 2> $O/bench_c${c}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_c${c}_$r.json').read().strip().splitlines()[-1]); print('bench c$c $r', d['value'], d['roofline']['frac'], {k: (v or {}).get('us_per_pair') for k, v in d['match_roofline'].items()})"
    grep -E "process_frame|extract wait|speculation wait" $O/bench_c${c}_$r.err
  done
done
echo done
