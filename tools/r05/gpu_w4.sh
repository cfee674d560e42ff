#!/bin/bash
# Round-5: F(4x4) on conv4a/b too (VS_WINO4_MIN_WG = 32 vs the default 64): network per layer, network error, headline
export TMPDIR=/tmp
O=gpurun_out/r05w4; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
for m in 64 32; do
  VS_WINO4_MIN_WG=$m timeout -k 10 300 python -u tools/bench_net.py --frames 8 --reps 20 > $O/net_$m.json 2> $O/net_$m.err || { tail -5 $O/net_$m.err; exit 1; }
  echo "min_wg $m net: $(tail -1 $O/net_$m.json | cut -c1-700)"
done
VS_WINO4_MIN_WG=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "network" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "network parity rc=$? $(tail -1 $O/pytest.log)"
for m in 64 32 64 32; do
  VS_WINO4_MIN_WG=$m timeout -k 10 400 python -u bench.py --no-cpu-baseline --ba-reps 0 --no-frontend --mono-steps 0 > $O/b_$m.json 2> $O/b_$m.err || { tail -5 $O/b_$m.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$m.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']
print('min_wg $m', d['value'], d['ms_per_step'], 'conv4a', s.get('conv4a'), 'conv4b', s.get('conv4b'))"
done
