#!/bin/bash
# Round-6 final: CU-partition knob A/B at HEAD (12-wave k_wino4): default vs the network off the speculative CUs,
# 16 speculative CUs, 24 / 40 tracking CUs; alternating, same box
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06kn}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py $H > $O/b_$tag.json 2> $O/b_$tag.err || { tail -20 $O/b_$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1])
print('$tag', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  run def$r VS_SLAM_X=0
  run netnone$r VS_SLAM_NET_SET=none
  run spec16$r VS_SLAM_SPEC_CUS=16
  run track24$r VS_SLAM_TRACK_CUS=24
  run track40$r VS_SLAM_TRACK_CUS=40
done
