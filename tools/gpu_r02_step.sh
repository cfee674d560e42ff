set -o pipefail
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_crmath.py > gpurun_out/t6a.log 2>&1 && \
timeout -k 10 120 python -u tools/bench_match.py --pairs 1,8,32,128,512 > gpurun_out/bm6.log 2>&1 && \
timeout -k 10 400 python -u tools/debug_tracker_divergence.py --loop 416 --batch 32 --tol 0 --after 2 --trace gpurun_out/tr6 > gpurun_out/div6.log 2>&1 ; \
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t6.log 2>&1
