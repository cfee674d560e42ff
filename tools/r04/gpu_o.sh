#!/bin/bash
# settle step: keyframe archiving and slot moves as one k_copy_jobs launch each (instead of ~50 memcpys per batch):
# tracker / loop-closure / dense parity, then headline A/B vs the committed HEAD build (ab/head.so)
export TMPDIR=/tmp
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_tracker.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker_ideal.py tests/test_gpu_tracking.py tests/test_gpu_stationary.py tests/test_gpu_dense.py tests/test_gpu_pgo.py tests/test_gpu_facade.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2; do
  for nl in old:ab/head.so new:visual-slam-pipeline_amd/libvslam_hip.so; do
    n=${nl%%:*}; lib=${nl#*:}
    VS_LIB_PATH=$lib VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); print('bench $n $r', d['value'], d['ate'].get('rank0_rmse_m'))"
    grep -E "process_frame" $O/bench_${n}_$r.err
  done
done
echo done
