export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
L=gpurun_out/s29.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_stationary.py > $L 2>&1
timeout -k 10 200 python -u tools/profile_tracker_phases.py > gpurun_out/phases29.json 2>> $L
timeout -k 10 800 python3 -u tools/cpu_baseline.py --frames 200 --threads 1 --out gpurun_out/cpu_baseline_1.json >> $L 2>&1
echo "exit $?" >> $L
