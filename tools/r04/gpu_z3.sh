#!/bin/bash
# speculative-chain CU count A/B at contiguous CU sets (VS_SLAM_SPEC_CUS 32 / 8 / 16 / 4): headline bench with the
# host profile, three rounds
export TMPDIR=/tmp
O=gpurun_out/r04z3; mkdir -p $O
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2 3; do
  for cfg in 32:32:0 32:8:0 32:16:0 32:4:0; do
    IFS=: read t sp spr <<< "$cfg"
    n=t${t}_s${sp}_x${spr}
    VS_SLAM_CU_SPREAD=$spr VS_SLAM_TRACK_CUS=$t VS_SLAM_SPEC_CUS=$sp VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); print('bench $n $r', d['value'], d['roofline']['frac'])"
    grep -E "process_frame|extract wait|speculation wait" $O/bench_${n}_$r.err
  done
done
echo done
