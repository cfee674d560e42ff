#!/bin/bash
# issue priority for the extraction post-processing waves (post_prio in sp_post.hip): post-processing parity,
# headline A/B vs the committed head (ab/head.so) with the host profile, three rounds
export TMPDIR=/tmp
O=gpurun_out/r04pp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2 3; do
  for nl in head:ab/head.so new:visual-slam-pipeline_amd/libvslam_hip.so; do
    n=${nl%%:*}; lib=${nl#*:}
    VS_LIB_PATH=$lib VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']; print('bench $n $r', d['value'], d['roofline']['frac'], s.get('nms_rounds'), s.get('nms_select'))"
    grep -E "process_frame|extract wait|speculation wait" $O/bench_${n}_$r.err
  done
done
echo done
