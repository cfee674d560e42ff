#!/bin/bash
# Round-6: EPnP out-of-line regression tests (B's diagonal by assignment); the default bench line; a 16-CU
# chain A/B; a kernel + HIP trace of the headline for the chain-wait analysis
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06m}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pnp.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|stage|differing" $O/pytest_pnp.log | tail -30
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
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/trace -o trace --output-format csv -- python3 bench.py $H > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 tools/r06/chain_wait.py $O/trace
python3 tools/trace_chain.py $(ls $O/trace/*kernel_trace.csv $O/trace/*/*kernel_trace.csv 2>/dev/null | head -1) > $O/chain.txt 2>&1; head -40 $O/chain.txt
[ $rc -eq 0 ] || echo "PNP TESTS FAILED"
