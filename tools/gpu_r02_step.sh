export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
L=gpurun_out/s27.log
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_midas.py -s > $L 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench27.json 2>> $L
echo "exit $?" >> $L
