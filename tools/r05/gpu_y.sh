#!/bin/bash
# Round-5: k_ba_chol_band without row tests + prefetched backward operands: parity, phases, A/B vs HEAD
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ba.py -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 tools/profile_ba_phases.py --span 3 > $O/phases_new.json 2> $O/phases.err || { tail -3 $O/phases.err; exit 1; }
cat $O/phases_new.json
for v in old new; do
  if [ $v = old ]; then export VS_LIB_PATH=tools/r05/ab/libvslam_old.so; else unset VS_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o ba --output-format csv -- \
      python3 tools/bench_ba.py --no-cpu --reps 5 > $O/ba_$v.log 2>&1 || { tail -5 $O/ba_$v.log; exit 1; }
  python3 - $O/prof_$v/ba_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'chol' in r['Name']:
        print(sys.argv[2], r['Name'][:40], 'calls', r['Calls'], 'avg_us %.1f' % (float(r['AverageNs']) / 1e3))
PY
  tail -1 $O/ba_$v.log | cut -c1-300
done
