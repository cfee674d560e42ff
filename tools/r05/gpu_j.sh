#!/bin/bash
# Round-5: k_pnp_hyp eigen-stage split (profiling build) + PnP / tracker parity
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pnp.py::test_epnp_sequential_device_equals_host tests/test_gpu_pnp.py tests/test_golden.py tests/test_gpu_tracker_ideal.py tests/test_gpu_tracker_bench.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; grep -E "passed|failed|Error" $O/pytest.log | tail -8; echo "pytest rc=$rc"
timeout -k 10 300 python -u tools/profile_tracker_phases.py > $O/phases.json 2> $O/phases.err || { tail -5 $O/phases.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/phases.json').read().strip().splitlines()[-1]); print('pnp phases', d.get('pnp_hyp_kcycles_per_hypothesis_x100'))"
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o tr --output-format csv -- python3 tools/bench_tracker.py --steps 6 > $O/tracker.log 2>&1 || { kill $HB; tail -5 $O/tracker.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r05j/prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('k_pnp', 'k_tlm', 'k_fmat', 'k_ransac3d', 'k_emat')):
        print('%-40s calls %6s avg_us %8.1f' % (r['Name'][:40], r['Calls'], float(r['AverageNs']) / 1e3))
PY
tail -3 $O/tracker.log
kill $HB
