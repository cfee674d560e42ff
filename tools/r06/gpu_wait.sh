#!/bin/bash
# Round-6: does the tracker thread pay interrupt wake-ups on its GPU waits?  Default vs ROC_ACTIVE_WAIT_TIMEOUT=1000
# (ROCclr spins that many us before blocking), alternating, same box; one host profile each
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06wt}; mkdir -p $O
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
for r in 1 2 3; do
  run def$r VS_X=0
  run spin$r ROC_ACTIVE_WAIT_TIMEOUT=1000
done
run hpdef VS_SLAM_HOST_PROFILE=1
grep "process_frame\|sync\|wait" $O/b_hpdef.err | head -8
run hpspin VS_SLAM_HOST_PROFILE=1 ROC_ACTIVE_WAIT_TIMEOUT=1000
grep "process_frame\|sync\|wait" $O/b_hpspin.err | head -8
