#!/bin/bash
# BA: banded Cholesky (k_ba_chol_band, one wave, S's band in LDS) vs the dense look-ahead kernel (VS_BA_BAND=0):
# BA parity and goldens, config[2] timing A/B, kernel trace
export TMPDIR=/tmp
O=gpurun_out/r04bb6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for bnd in 1 0; do
    VS_BA_BAND=$bnd VS_BA_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 5 > $O/bench_b${bnd}_$r.json 2> $O/bench_b${bnd}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_b${bnd}_$r.json').read().strip().splitlines()[-1]); b=d['local_ba']; print('ba band=$bnd', b['ms_per_call'], b['ms_per_iteration'], b['lm_iterations'], b['rms_after'], b['stage_ms_per_call'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 3 --render-workers 1 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); grep -E "k_ba_" $f | cut -d, -f1-4; cp $f $O/ba_kernel_stats.csv
rm -f $(find $O/prof -name "*kernel_trace.csv")
echo done
