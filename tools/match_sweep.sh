#!/bin/bash
# Matcher tile / phase sweep on one GPU: bit-exactness of every tile variant (the match parity
# tests under VS_MATCH_TILE), then rocprofv3 kernel durations of tools/bench_match.py per variant
# and per phase ablation (VS_MATCH_ABLATE 1: stop after the k-loop, 2: no MFMAs, 3: prologue only).
export TMPDIR=/tmp
OUT=gpurun_out/match_sweep
mkdir -p $OUT
for t in ${TILES:-q32t32 q32t64 q64t32 w8 w8k64}; do
  VS_MATCH_TILE=$t timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "match" -p no:cacheprovider \
      > $OUT/parity_$t.log 2>&1 || { echo "parity $t FAILED"; tail -20 $OUT/parity_$t.log; exit 1; }
  echo "parity $t ok"
done
for t in default ${TILES:-q32t32 q32t64 q64t32 w8 w8k64} k64 small; do
  for abl in 0 ${ABLS:-}; do
    tag=${t}_a${abl}
    VS_MATCH_TILE=$t VS_MATCH_ABLATE=$abl timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o m \
        --output-format csv -- python3 tools/bench_match.py --pairs ${PAIRS:-1,32,512} --reps 20 > $OUT/$tag.log 2>&1 \
        || { echo "bench $tag FAILED"; tail -5 $OUT/$tag.log; exit 1; }
    echo "bench $tag ok"
  done
done
