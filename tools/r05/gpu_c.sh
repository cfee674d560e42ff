#!/bin/bash
# Round-5: k_wino4 latency ablation (builds whose results are wrong by construction; abl/libabl<N>.so)
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
for v in base 1 2 3 4 5 base; do
  if [ $v = base ]; then L=""; else L=$PWD/abl/libabl$v.so; fi
  VS_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_net.py --reps 10 --frames 8 > $O/bench_net_$v.json 2> $O/bench_net_$v.err || { tail -20 $O/bench_net_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_net_$v.json').read().strip().splitlines()[-1])
l = d['frames_8']['layers']
print('abl=$v', d['frames_8']['network_ms_per_launch'], {n: l[n]['ms_per_launch'] for n in ('conv1_fused','conv2a','conv2b_pool','conv3a','conv3b_pool','head_a')})"
done
echo done
