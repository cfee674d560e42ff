#!/bin/bash
# Round-6: two network streams, each chunk started once the previous one passed its early layers: parity, A/B
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline_drive.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" $O/pytest.log | tail -3
[ $rc -eq 0 ] || exit 1
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for t in 2 1 2 1; do
  VS_SLAM_NET_STREAMS=$t timeout -k 10 300 python -u bench.py $H > $O/b_$t.json 2> $O/b_$t.err || { tail -20 $O/b_$t.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']
net=sum(v for k,v in s.items() if k.startswith('conv') or k.startswith('head') or k=='gray_norm')
print('streams=$t', d['value'], d['ms_per_step'], 'net/frame %.4f' % net, 'conv1', d['roofline']['avg_launch_ms'])"
done
for ov in 2 4 1; do
  VS_SLAM_NET_OVERLAP=$ov timeout -k 10 300 python -u bench.py $H > $O/b_ov$ov.json 2> $O/b_ov$ov.err || { tail -20 $O/b_ov$ov.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_ov$ov.json').read().strip().splitlines()[-1])
print('overlap=$ov', d['value'], d['ms_per_step'], 'conv1', d['roofline']['avg_launch_ms'])"
done
