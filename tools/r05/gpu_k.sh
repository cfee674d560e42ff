#!/bin/bash
# Round-5: headline + chain trace after the EPnP rewrite: bench line (no CPU baseline), host profile of
# process_frame, rocprofv3 kernel trace of the tracker-only bench and the chain summary
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
timeout -k 10 900 python -u bench.py --no-cpu-baseline --ba-reps 0 > $O/bench.json 2> $O/bench.err || { kill $HB; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); fe=d['frontend_batch']; m=d['match_roofline']
print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['map_points'], d['keyframes'])
print('stage', json.dumps(d['stage_ms_per_frame']))
print('fe', fe['value'], fe['ms_per_step'], 'match fe', m['frontend_batch']['frac'], 'tracker match', json.dumps({k: v for k, v in m.items() if k != 'frontend_batch'})[:400])
print('mono', d['monocular_hd']['value'])"
VS_SLAM_HOST_PROFILE=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --ba-reps 0 --no-frontend --mono-steps 0 > $O/bench_hp.json 2> $O/bench_hp.err || { kill $HB; tail -20 $O/bench_hp.err; exit 1; }
grep -E "process_frame|track_local_map|solve_pnp|chain" $O/bench_hp.err | tail -12
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --render-workers 1 --ba-reps 0 > $O/prof.log 2>&1 || { kill $HB; tail -5 $O/prof.log; exit 1; }
python3 tools/trace_chain.py $(ls $O/prof/*/trace_kernel_trace.csv $O/prof/trace_kernel_trace.csv 2>/dev/null | head -1) > $O/chain.txt 2>&1; tail -30 $O/chain.txt
kill $HB
echo done
