#!/bin/bash
# Round-6: convDb + convPb (1x1 heads) in one grid (k_conv1x1_pair) vs two launches (previous library):
# network parity, network alone, headline alternating x3
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06hb}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "network or extract" > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2
[ $rc -eq 0 ] || exit 1
for t in new old; do
  L=""; [ $t = old ] && L=$PWD/tools/r06/oldlib/libvslam_hip.so
  VS_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_net.py --frames 8,32 --reps 10 > $O/net_$t.json 2> $O/net_$t.err || { tail $O/net_$t.err; exit 1; }
  python3 -c "
import json
for l in open('$O/net_$t.json'):
    try: d=json.loads(l)
    except Exception: continue
    L=d['frames_8']['layers']; print('$t', {k: v['ms_per_launch'] for k, v in L.items()})"
done
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for t in new old new old new old; do
  L=""; [ $t = old ] && L=$PWD/tools/r06/oldlib/libvslam_hip.so
  VS_LIB_PATH=$L timeout -k 10 300 python -u bench.py $H > $O/b_$t.json 2> $O/b_$t.err || { tail -20 $O/b_$t.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']
net=sum(v for k,v in s.items() if k.startswith('conv') or k.startswith('head') or k=='gray_norm')
print('$t', d['value'], d['ms_per_step'], 'net/frame %.4f' % net, 'conv1', d['roofline']['avg_launch_ms'], 'spec', s.get('match_spec'), s.get('fmat_ransac'))"
done
