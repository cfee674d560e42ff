#!/bin/bash
# EPnP Jacobi variant 2 (each round's 6 angles computed once on lanes 36..41, read from LDS) vs HEAD:
# parity of the variant build, PnP phase cycles and k_pnp_hyp durations of both
export TMPDIR=/tmp
O=gpurun_out/r04q; mkdir -p $O
VS_LIB_PATH=ab/j2.so timeout -k 10 900 python -u -m pytest tests/test_gpu_pnp.py tests/test_golden.py tests/test_gpu_tracker.py tests/test_gpu_tracker_bench.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in head:visual-slam-pipeline_amd/libvslam_hip_prof.so j2:ab/j2_prof.so; do
  n=${v%%:*}; lib=${v#*:}
  VS_PROF_LIB=$lib timeout -k 10 300 python -u tools/profile_tracker_phases.py > $O/phases_$n.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/phases_$n.log').read().strip().splitlines()[-1]); print('$n', d['pnp_hyp_kcycles_per_hypothesis_x100'])"
done
for v in head:visual-slam-pipeline_amd/libvslam_hip.so j2:ab/j2.so; do
  n=${v%%:*}; lib=${v#*:}
  VS_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o trace --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --render-workers 1 > $O/prof_$n.log 2>&1 || exit 1
  f=$(find $O/prof_$n -name "*kernel_stats.csv" | head -1); echo "$n $(grep -E 'k_pnp_hyp' $f | cut -d, -f2-4)"
done
echo done
