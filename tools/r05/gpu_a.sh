#!/bin/bash
# Round-5: F(4x4,3x3) first light — network error vs torch fp64 and the network alone per layer, F2 vs F4
export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
for v in 0 1; do
  VS_WINO4=$v timeout -k 10 300 python -u tools/net_err.py > $O/net_err_$v.json 2> $O/net_err_$v.err || { tail -20 $O/net_err_$v.err; exit 1; }
  echo "wino4=$v"; cat $O/net_err_$v.json
done
for v in 0 1 0 1; do
  VS_WINO4=$v timeout -k 10 300 python -u tools/bench_net.py --reps 10 > $O/bench_net_$v.json 2> $O/bench_net_$v.err || { tail -20 $O/bench_net_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_net_$v.json').read().strip().splitlines()[-1])
for k in ('frames_8','frames_32'):
    print('wino4=$v', k, d[k]['network_ms_per_launch'], {n: v['ms_per_launch'] for n, v in d[k]['layers'].items()})"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.log 2>&1; tail -3 $O/pytest_parity.log
echo done
