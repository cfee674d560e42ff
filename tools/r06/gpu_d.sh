#!/bin/bash
# Round-6: local-map tracking without the grid kernel (grid built at extraction) and with the PnP gather
# fused into k_tlm_resolve: tracker / TLM parity, the new batch-vs-oracle and out-of-line EPnP tests, bench
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06d}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline_drive.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py tests/test_gpu_tracking.py tests/test_gpu_stationary.py tests/test_golden.py tests/test_gpu_batch.py tests/test_gpu_pnp.py -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|mode . differing|pairs:" $O/pytest.log | tail -40
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
VS_SLAM_PRE_GRID=0 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 > $O/bench_nopre.json 2> $O/bench_nopre.err || { tail -20 $O/bench_nopre.err; exit 1; }
VS_SLAM_HOST_PROFILE=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 > $O/bench_hp.json 2> $O/bench_hp.err || { tail -20 $O/bench_hp.err; exit 1; }
grep "vs_slam" $O/bench_hp.err | head -20
python3 -c "
import json
for n in ('bench', 'bench_nopre', 'bench_hp'):
    d=json.loads(open('$O/%s.json' % n).read().strip().splitlines()[-1])
    print(n, d['value'], d['ms_per_step'], d['stage_ms_per_frame'].get('track_local_map'), d['stage_ms_per_frame'].get('solve_pnp'))"
