#!/bin/bash
# Round-5: k_wino4 with conv1a on the matrix cores (conv1): error, network per layer, parity subset
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 300 python -u tools/net_err.py > $O/net_err.json 2> $O/net_err.err || { tail -20 $O/net_err.err; exit 1; }
cat $O/net_err.json
for v in 1 1; do
  VS_WINO4=$v timeout -k 10 300 python -u tools/bench_net.py --reps 10 > $O/bench_net_$v.json 2> $O/bench_net_$v.err || { tail -20 $O/bench_net_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_net_$v.json').read().strip().splitlines()[-1])
for k in ('frames_8','frames_32'):
    print('wino4=$v', k, d[k]['network_ms_per_launch'], {n: v['ms_per_launch'] for n, v in d[k]['layers'].items()})"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_monocular.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.log 2>&1; tail -3 $O/pytest_parity.log
echo done
