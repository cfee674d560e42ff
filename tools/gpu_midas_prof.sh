#!/bin/bash
# MiDaS alone: ms per 32-frame batch with VS_WINO=0 / 1, then a rocprofv3 kernel trace (per-kernel split).
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
for w in 0 1; do
  VS_WINO=$w timeout -k 10 200 python -u tools/bench_midas.py > $O/midas_w$w.json 2> $O/midas_w$w.err || exit 1
  echo "wino=$w $(tail -1 $O/midas_w$w.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o midas --output-format csv -- \
    python3 tools/bench_midas.py --reps 5 > $O/prof.log 2>&1 || exit 1
echo prof ok
