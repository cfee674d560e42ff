export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
L=gpurun_out/s20.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tracker.py tests/test_gpu_tracker_bench.py > $L 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 > gpurun_out/bench20.json 2>> $L &&
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 > gpurun_out/bench20_hprof.json 2>> $L
echo "exit $?" >> $L
