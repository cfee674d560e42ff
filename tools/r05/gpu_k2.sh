#!/bin/bash
# Round-5: stream / CU-set knobs after conv4's F(4x4) (headline only): the network or the post-processing also on the
# speculative chain's CUs, 32-channel chunks in the 1x1 heads
export TMPDIR=/tmp
O=gpurun_out/r05k2; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
run() {  # name, then env assignments
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --no-cpu-baseline --ba-reps 0 --no-frontend --mono-steps 0 > $O/b_$name.json 2> $O/b_$name.err || { tail -5 $O/b_$name.err; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'])"
}
run default VS_DUMMY=1 && run net_spec VS_SLAM_NET_SET=spec && run post_spec VS_SLAM_POST_SET=spec && run ck32 VS_CONV1X1_CK=32 && run default2 VS_DUMMY=1 && run net_spec2 VS_SLAM_NET_SET=spec
