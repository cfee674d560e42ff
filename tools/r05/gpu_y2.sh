#!/bin/bash
# Round-5: band Cholesky backward select order + the dense kernel on a non-banded window (span 8)
export TMPDIR=/tmp
O=gpurun_out/r05y2; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ba.py -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 tools/profile_ba_phases.py --span 3 > $O/phases.json 2> $O/phases.err || { tail -3 $O/phases.err; exit 1; }
cat $O/phases.json
for sp in 3 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_s$sp -o ba --output-format csv -- \
      python3 tools/bench_ba.py --no-cpu --reps 5 --span $sp > $O/ba_s$sp.log 2>&1 || { tail -5 $O/ba_s$sp.log; exit 1; }
  python3 - $O/prof_s$sp/ba_kernel_stats.csv $sp <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_ba' in r['Name']:
        print('span', sys.argv[2], '%-36s calls %5s avg_us %8.1f' % (r['Name'][:36], r['Calls'], float(r['AverageNs']) / 1e3))
PY
  tail -1 $O/ba_s$sp.log | cut -c1-400
done
