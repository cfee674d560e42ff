#!/bin/bash
# BA (look-ahead Cholesky, LM enqueue stop) + branch-free sym_eig (Kabsch / control / triangulation):
# parity, BA / PnP phases, config[2] timing, headline A/B vs ab/tlm.so
export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ba.py tests/test_golden.py tests/test_gpu_pnp.py tests/test_gpu_emat.py tests/test_gpu_tracking.py tests/test_gpu_tracker.py tests/test_gpu_tracker_ideal.py tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/profile_ba_phases.py > $O/ba_phases.log 2>&1 || exit 1; tail -1 $O/ba_phases.log
timeout -k 10 300 python -u tools/profile_tracker_phases.py > $O/phases.log 2>&1 || exit 1; python3 -c "import json; d=json.loads(open('$O/phases.log').read().strip().splitlines()[-1]); print(d['pnp_hyp_kcycles_per_hypothesis_x100'])"
VS_BA_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 5 > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); b=d['local_ba']; print('head', d['value'], 'ba', b['ms_per_call'], b['ms_per_iteration'], b['lm_iterations'], b['stage_ms_per_call'], 'pnp', d['stage_ms_per_frame'].get('solve_pnp'))"
grep "vs_local_ba host" $O/bench.err | tail -1
VS_LIB_PATH=ab/tlm.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 5 > $O/bench_old.json 2> $O/bench_old.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench_old.json').read().strip().splitlines()[-1]); b=d['local_ba']; print('old', d['value'], 'ba', b['ms_per_call'], b['ms_per_iteration'], b['lm_iterations'], b['stage_ms_per_call'], 'pnp', d['stage_ms_per_frame'].get('solve_pnp'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 3 --render-workers 1 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); grep -E "k_ba_chol|k_pnp_hyp|k_pnp_ransac|k_match" $f | cut -d, -f1-4
echo done
