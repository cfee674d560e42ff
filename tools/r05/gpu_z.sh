#!/bin/bash
# Round-5: PnP solver changes (the unscaled division / sqrt experiment; the LM pivot reciprocals): probe, parity, kernel A/B
export TMPDIR=/tmp
O=gpurun_out/${GPU_Z_OUT:-r05z}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 tools/r05/rsq_exact > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracking.py tests/test_gpu_tracker.py tests/test_golden.py tests/test_gpu_ba.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; grep -E "^FAILED|passed|failed" $O/pytest.log | tail -8
tail -1 $O/pytest.log
ARGS="--steps 4 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --render-workers 1 --ba-reps 0"
for v in old new; do
  if [ $v = old ]; then export VS_LIB_PATH=tools/r05/ab/libvslam_old.so; else unset VS_LIB_PATH; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o trk --output-format csv -- python3 bench.py $ARGS > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python3 - $O/prof_$v/trk_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r['Name'] for k in ('k_pnp', 'k_fmat', 'k_ransac3d', 'k_emat', 'k_tlm')):
        print(sys.argv[2], '%-34s calls %6s avg_us %8.1f' % (r['Name'][:34], r['Calls'], float(r['AverageNs']) / 1e3))
PY
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', 'fps', d['value'])"
done
