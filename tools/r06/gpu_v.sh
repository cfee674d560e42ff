#!/bin/bash
# Round-6: band Cholesky backward substitution with a 3-deep L prefetch and deferred x stores: BA parity,
# config[2] timing vs the previous library, phase cycles (profiling build)
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" $O/pytest.log | tail -3
[ $rc -eq 0 ] || exit 1
for t in new old new old; do
  L=""; [ $t = old ] && L=$PWD/tools/r06/oldlib/libvslam_hip.so
  VS_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_ba.py --reps 5 --no-cpu > $O/ba_$t.json 2> $O/ba_$t.err || { tail $O/ba_$t.err; exit 1; }
  echo "$t $(tail -c 600 $O/ba_$t.json)"
done
timeout -k 10 300 python -u tools/profile_ba_phases.py > $O/ba_phases.json 2> $O/ba_phases.err && cat $O/ba_phases.json | head -c 1500
