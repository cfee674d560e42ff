#!/bin/bash
# Round-5: k_ba_chol_band A/B (HEAD library vs the working tree), config[2] window, BA parity
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
for v in old new; do
  if [ $v = old ]; then export VS_LIB_PATH=tools/r05/ab/libvslam_old.so; else unset VS_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o ba --output-format csv -- \
      python3 tools/bench_ba.py --no-cpu --reps 5 > $O/ba_$v.log 2>&1 || { tail -5 $O/ba_$v.log; exit 1; }
done
unset VS_LIB_PATH
for v in old new; do
  python3 - $O/prof_$v/ba_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'chol' in r['Name']:
        print(sys.argv[2], r['Name'][:40], 'calls', r['Calls'], 'avg_us %.1f' % (float(r['AverageNs']) / 1e3))
PY
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $O/pytest.log
