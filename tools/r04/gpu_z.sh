#!/bin/bash
# CU partition sweep at HEAD (the tracker now waits for the network at chunk boundaries): VS_SLAM_TRACK_CUS /
# VS_SLAM_SPEC_CUS / VS_SLAM_POST_SET / VS_SLAM_NET_SET, headline bench with the host profile, two rounds
export TMPDIR=/tmp
O=gpurun_out/r04z; mkdir -p $O
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2; do
  for cfg in 32:32:-:- 32:16:-:- 32:24:-:- 24:24:-:- 32:8:-:- 32:32:track:- 32:32:-:spec 32:32:-:all; do
    IFS=: read t sp ps ns <<< "$cfg"
    n=t${t}_s${sp}_${ps}_${ns}
    if [ "$ps" = "-" ]; then unset VS_SLAM_POST_SET; else export VS_SLAM_POST_SET=$ps; fi
    if [ "$ns" = "-" ]; then unset VS_SLAM_NET_SET; else export VS_SLAM_NET_SET=$ns; fi
    VS_SLAM_TRACK_CUS=$t VS_SLAM_SPEC_CUS=$sp VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); print('bench $n $r', d['value'], d['roofline']['frac'])"
    grep -E "process_frame|extract wait|speculation wait" $O/bench_${n}_$r.err
  done
done
echo done
