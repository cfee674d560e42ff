#!/bin/bash
# the speculative chain on the network's CUs (VS_SLAM_SPEC_CUS=0 VS_SLAM_SPEC_SET=net: the network keeps seven whole
# XCDs) vs its own 8 CUs, and on the tracking CUs (SPEC_CUS=0): headline bench with the host profile, three rounds
export TMPDIR=/tmp
O=gpurun_out/r04z5; mkdir -p $O
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2 3; do
  for cfg in 8:- 0:net 0:-; do
    IFS=: read sp ss <<< "$cfg"
    n=s${sp}_${ss}
    if [ "$ss" = "-" ]; then unset VS_SLAM_SPEC_SET; else export VS_SLAM_SPEC_SET=$ss; fi
    VS_SLAM_SPEC_CUS=$sp VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); print('bench $n $r', d['value'], d['roofline']['frac'])"
    grep -E "process_frame|extract wait|speculation wait" $O/bench_${n}_$r.err
  done
done
echo done
