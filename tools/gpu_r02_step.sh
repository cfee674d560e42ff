export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
L=gpurun_out/s15.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tracker.py tests/test_gpu_spcf.py tests/test_gpu_facade.py > $L 2>&1 || { echo "exit tests" >> $L; exit 1; }
for v in default t80q t64; do
  if [ $v = default ]; then unset VS_MATCH_TILE; else export VS_MATCH_TILE=$v; fi
  echo "== $v" >> $L
  timeout -k 10 120 python -u tools/bench_match.py --pairs 1,8,32,128,512 >> $L 2>&1 || exit 1
done
unset VS_MATCH_TILE
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof15 -o m --output-format csv -- python3 -u tools/bench_match.py --pairs 1,32,512 --reps 20 >> $L 2>&1
echo "exit $?" >> $L
