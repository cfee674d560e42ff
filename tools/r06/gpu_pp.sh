#!/bin/bash
# Round-6: post-processing CU set A/B at HEAD
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06pp}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py $H > $O/b_$n.json 2> $O/b_$n.err || { tail -20 $O/b_$n.err; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$n.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']
net=sum(v for k,v in s.items() if k.startswith('conv') or k.startswith('head') or k=='gray_norm')
print('$n', d['value'], d['ms_per_step'], 'net/frame %.4f' % net, 'conv1', d['roofline']['avg_launch_ms'])"
}
run base VS_X=0 &&
run ptrack VS_SLAM_POST_SET=track &&
run pc8 VS_SLAM_POST_CUS=8 &&
run pc16 VS_SLAM_POST_CUS=16 &&
run base2 VS_X=0 &&
run ptrack2 VS_SLAM_POST_SET=track
