#!/bin/bash
# Round-6: host timeline of the tracker thread (rocprofv3 HIP API + kernel trace of the tracker-only bench)
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06c}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 6 --warmup 1 --track-profile-steps 0 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --render-workers 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
ls -R $O/prof | head
python3 tools/r06/host_timeline.py $O/prof > $O/host_timeline.txt 2>&1; cat $O/host_timeline.txt
python3 tools/trace_chain.py $(ls $O/prof/*/trace_kernel_trace.csv $O/prof/trace_kernel_trace.csv 2>/dev/null | head -1) > $O/chain.txt 2>&1; head -30 $O/chain.txt
# k_wino4 fixed per-workgroup cost: the network alone with half the k-steps (abl 6) and two k-steps (abl 7)
for v in base 6 7; do
  if [ $v = base ]; then L=""; else L=$PWD/abl/libabl$v.so; fi
  VS_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_net.py --reps 10 --frames 8 > $O/bench_net_$v.json 2> $O/bench_net_$v.err || { tail -20 $O/bench_net_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_net_$v.json').read().strip().splitlines()[-1])
l = d['frames_8']['layers']
print('abl=$v', d['frames_8']['network_ms_per_launch'], {n: l[n]['ms_per_launch'] for n in l})"
done
