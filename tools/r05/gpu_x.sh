#!/bin/bash
# Round-5: k_ba_chol_band scheduling variants (loads before the pivot chain, sched barriers, fence), A/B + parity
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
for v in old sb0_f1 sb1_f1 sb1_f0 sb2_f0 sb0_f0; do
  export VS_LIB_PATH=tools/r05/ab/libvslam_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o ba --output-format csv -- \
      python3 tools/bench_ba.py --no-cpu --reps 5 > $O/ba_$v.log 2>&1 || { tail -5 $O/ba_$v.log; exit 1; }
  python3 - $O/prof_$v/ba_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'chol' in r['Name']:
        print(sys.argv[2], r['Name'][:40], 'calls', r['Calls'], 'avg_us %.1f' % (float(r['AverageNs']) / 1e3))
PY
  timeout -k 10 200 python -u -m pytest tests/test_gpu_ba.py -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1; echo "$v pytest rc=$?"
done
