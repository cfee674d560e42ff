#!/bin/bash
# BA: next trailing tile prefetched in the look-ahead round
export TMPDIR=/tmp
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/profile_ba_phases.py > $O/ba_phases.log 2>&1 || exit 1; tail -1 $O/ba_phases.log
for r in 1 2; do
VS_BA_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 5 > $O/bench_$r.json 2> $O/bench_$r.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench_$r.json').read().strip().splitlines()[-1]); b=d['local_ba']; print('ba', b['ms_per_call'], b['ms_per_iteration'], b['lm_iterations'], b['stage_ms_per_call'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 3 --render-workers 1 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); grep -E "k_ba_" $f | cut -d, -f1-4
echo done
# (result: slower — diag_ahead+trailing 355 -> 410 kcycles, config[2] 4.67 -> 4.86 ms; the prefetch spilled registers; reverted)
