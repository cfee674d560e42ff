#!/bin/bash
# Round-6: k_wino4 on 16 waves (3 x 3 domain quarters, 4 waves per SIMD) vs 12 (row pairs): parity under
# VS_WINO4_XG=4, network alone, headline A/B alternating
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06xg4}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
VS_WINO4_XG=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "network or extract" > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
for v in 4 3; do
  VS_WINO4_XG=$v timeout -k 10 300 python -u tools/bench_net.py --frames 8,32 --reps 10 > $O/net_$v.json 2> $O/net_$v.err || { tail $O/net_$v.err; exit 1; }
  python3 -c "
import json
for l in open('$O/net_$v.json'):
    try: d=json.loads(l)
    except Exception: continue
    L=d['frames_8']['layers']; print('xg=$v', {k: v['ms_per_launch'] for k, v in L.items()})"
done
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for v in 4 3 4 3; do
  VS_WINO4_XG=$v timeout -k 10 300 python -u bench.py $H > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']
net=sum(v for k,v in s.items() if k.startswith('conv') or k.startswith('head') or k=='gray_norm')
print('xg=$v', d['value'], d['ms_per_step'], 'net/frame %.4f' % net, 'conv1', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
