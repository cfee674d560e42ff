#!/bin/bash
# Round-6: static-index Jacobi (sym_eig_static) in EPnP's control points, Kabsch and the DLT: the PnP / 3D-3D /
# tracker suites, then the headline A/B against the HEAD library (tools/r06/oldlib) alternating
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06se}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_tracker.py tests/test_gpu_tracking.py tests/test_gpu_stationary.py tests/test_gpu_headline_drive.py tests/test_gpu_tracker_bench.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $O/pytest.log | tail -5
[ $rc -eq 0 ] || exit 1
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for t in new old new old; do
  L=""; [ $t = old ] && L=$PWD/tools/r06/oldlib/libvslam_hip.so
  VS_LIB_PATH=$L timeout -k 10 300 python -u bench.py $H > $O/b_$t.json 2> $O/b_$t.err || { tail -20 $O/b_$t.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']
print('$t', d['value'], d['ms_per_step'], 'pnp', s.get('solve_pnp'), 'tlm', s.get('track_local_map'), 'r3d', s.get('ransac3d'), 'fmat', s.get('fmat_ransac'))"
done
