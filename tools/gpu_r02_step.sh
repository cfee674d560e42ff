export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
L=gpurun_out/s33.log
timeout -k 10 60 ./tools/crlat > $L 2>&1 &&
timeout -k 10 700 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_crmath.py tests/test_gpu_tracker_bench.py -m gpu >> $L 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 > gpurun_out/bench33.json 2>> $L &&
timeout -k 10 200 python -u tools/profile_tracker_phases.py > gpurun_out/phases33.json 2>> $L
echo "exit $?" >> $L
