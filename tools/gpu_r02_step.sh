export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
L=gpurun_out/s12.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu > $L 2>&1 &&
for v in shallow deep auto; do
  if [ $v = auto ]; then unset VS_MATCH_TILE; else export VS_MATCH_TILE=$v; fi
  echo "== $v" >> $L
  timeout -k 10 120 python -u tools/bench_match.py --pairs 1,2,4,8,32,512 >> $L 2>&1 || exit 1
done &&
unset VS_MATCH_TILE &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 >> $L 2>&1
echo "exit $?" >> $L
