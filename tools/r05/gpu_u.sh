#!/bin/bash
# Round-5: PMC bytes of the fused post-processing (tracker-only bench, one 8-frame chunk per launch)
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
PMC_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --render-workers 1 --ba-reps 0"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/prof_fetch -o fetch --output-format csv -- \
    python3 bench.py $PMC_ARGS > $O/prof_fetch.log 2>&1 && echo "fetch ok" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/prof_write -o write --output-format csv -- \
    python3 bench.py $PMC_ARGS > $O/prof_write.log 2>&1 && echo "write ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_post -o post --output-format csv -- \
    python3 tools/bench_post.py --batch 8 --reps 40 > $O/prof_post.log 2>&1 && echo "post trace ok"
