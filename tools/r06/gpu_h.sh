#!/bin/bash
# Round-6: k_wino4p (persistent runs of blocks): bit-exactness vs k_wino4 and the network tests, the network
# alone per run length, the headline with run = default vs 0
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06h}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 tools/r06/epnp_b_repro > $O/epnp_b_repro.txt 2>&1; cat $O/epnp_b_repro.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline_drive.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py -m gpu -v -s -k "network or headline or bench_scale or tracker" --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
for r in 0 2 4 8 0 2 4 8; do
  VS_WINO4_RUN=$r timeout -k 10 300 python -u tools/bench_net.py --reps 10 --frames 8,32 > $O/bench_net_r$r.json 2> $O/bench_net_r$r.err || { tail -20 $O/bench_net_r$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_net_r$r.json').read().strip().splitlines()[-1])
for f in ('frames_8', 'frames_32'):
    l = d[f]['layers']
    print('run=$r', f, d[f]['network_ms_per_launch'], {n: l[n]['ms_per_launch'] for n in ('conv1_fused', 'conv2a', 'conv2b_pool', 'conv3b_pool', 'head_a')})"
done
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $H > $O/bench_hp.json 2> $O/bench_hp.err || { tail -20 $O/bench_hp.err; exit 1; }
grep "vs_slam" $O/bench_hp.err | head -24
for r in -1 0 -1 0; do
  if [ $r = -1 ]; then E=""; else E="VS_WINO4_RUN=$r"; fi
  env $E timeout -k 10 300 python -u bench.py $H > $O/bench_r$r.json 2> $O/bench_r$r.err || { tail -20 $O/bench_r$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_r$r.json').read().strip().splitlines()[-1])
print('headline run=$r', d['value'], d['ms_per_step'], 'conv1', d['roofline']['avg_launch_ms'], d['roofline']['frac'], 'net', sum(v for k, v in d['stage_ms_per_frame'].items() if k.startswith(('conv', 'head'))))"
done
