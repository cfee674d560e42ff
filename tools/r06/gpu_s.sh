#!/bin/bash
# Round-6: (k_wino4 epilogue skew) CU-set combinations around "network also on the speculative chain's CUs" (same box, in-tree library)
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06s}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "network or extract" > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -u tools/bench_net.py --frames 8,32 --reps 10 > $O/net.json 2> $O/net.err && grep -o '"conv1_fused": {"ms_per_launch": [0-9.]*' $O/net.json | head -2
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
run ns VS_SLAM_NET_SET=spec &&
run ns_t24 VS_SLAM_NET_SET=spec VS_SLAM_TRACK_CUS=24 &&
run ns_ch16 VS_SLAM_NET_SET=spec VS_SLAM_CHUNK=16 &&
run ns_s16 VS_SLAM_NET_SET=spec VS_SLAM_SPEC_CUS=16 &&
run ns_s16_t24 VS_SLAM_NET_SET=spec VS_SLAM_SPEC_CUS=16 VS_SLAM_TRACK_CUS=24 &&
run ns_t24_ch16 VS_SLAM_NET_SET=spec VS_SLAM_TRACK_CUS=24 VS_SLAM_CHUNK=16 &&
run ns_d1 VS_SLAM_NET_SET=spec VS_SLAM_SPEC_DEPTH=1 &&
run ns2 VS_SLAM_NET_SET=spec &&
run base2 VS_X=0
