export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tracker.py tests/test_gpu_tracker_bench.py tests/test_gpu_parity.py -k "match or tracker" > gpurun_out/t9.log 2>&1
echo "tests exit $?" >> gpurun_out/t9.log
for v in default large2 small; do
  if [ $v = default ]; then unset VS_MATCH_TILE; else export VS_MATCH_TILE=$v; fi
  echo "== $v" >> gpurun_out/bm9.log
  timeout -k 10 120 python -u tools/bench_match.py --pairs 1,8,32,128,512 >> gpurun_out/bm9.log 2>&1 || break
done
unset VS_MATCH_TILE
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --frontend-steps 0 --mono-steps 0 > gpurun_out/bench9a.log 2>&1
VS_MATCH_TILE=large timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --frontend-steps 0 --mono-steps 0 > gpurun_out/bench9b.log 2>&1
echo done
