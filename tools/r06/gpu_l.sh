#!/bin/bash
# Round-6: EPnP out-of-line repro (if-assignment / copied R^T variants); the default bench line (front end on
# the drive's distinct frames) and a 16-CU chain A/B
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06l}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 tools/r06/epnp_b_repro > $O/epnp_b_repro.txt 2>&1; tail -7 $O/epnp_b_repro.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], 'fe', d['frontend_batch']['value'], d['frontend_batch'].get('ms_per_step'), 'mono', d['monocular_hd']['value'])"
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for c in 16 8 16 8; do
  VS_SLAM_SPEC_CUS=$c timeout -k 10 300 python -u bench.py $H > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -20 $O/bench_c$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_c$c.json').read().strip().splitlines()[-1])
print('spec_cus=$c', d['value'], d['ms_per_step'])"
done
