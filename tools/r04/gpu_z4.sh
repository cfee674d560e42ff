#!/bin/bash
# tracking + speculative-chain CUs inside one XCD (network on the other seven) vs 32 + 8: headline bench with the
# host profile, two rounds
export TMPDIR=/tmp
O=gpurun_out/r04z4; mkdir -p $O
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2; do
  for cfg in 32:8:0 28:4:0 26:6:0 28:8:0 25:7:0; do
    IFS=: read t sp spr <<< "$cfg"
    n=t${t}_s${sp}_x${spr}
    VS_SLAM_CU_SPREAD=$spr VS_SLAM_TRACK_CUS=$t VS_SLAM_SPEC_CUS=$sp VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); print('bench $n $r', d['value'], d['roofline']['frac'])"
    grep -E "process_frame|extract wait|speculation wait" $O/bench_${n}_$r.err
  done
done
echo done
