#!/bin/bash
# Round-6 final (B): rocprofv3 passes over the default-config bench (tools/profile_gpu.sh: kernel trace + stats,
# FETCH_SIZE, WRITE_SIZE, MFMA busy, matcher alone) and the post-processing trace pass of VERDICT r05 #10
export TMPDIR=/tmp
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
bash tools/profile_gpu.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_post -o post --output-format csv -- \
    python3 tools/bench_post.py --batch 8 --reps 40 > gpurun_out/prof_post.log 2>&1 && echo "post trace ok"
