#!/bin/bash
# the extraction post-processing stream on the speculative chain's 8 CUs (VS_SLAM_POST_SET=spec) or the tracking CUs
# (track) instead of the network's: headline bench with the host profile, three rounds
export TMPDIR=/tmp
O=gpurun_out/r04z6; mkdir -p $O
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2 3; do
  for ps in - spec track; do
    n=p_${ps}
    if [ "$ps" = "-" ]; then unset VS_SLAM_POST_SET; else export VS_SLAM_POST_SET=$ps; fi
    VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']; print('bench $n $r', d['value'], d['roofline']['frac'], s.get('nms_rounds'), s.get('nms_select'))"
    grep -E "process_frame|extract wait|speculation wait" $O/bench_${n}_$r.err
  done
done
echo done
