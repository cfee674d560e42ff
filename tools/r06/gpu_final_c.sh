#!/bin/bash
# Round-6 final profiles at HEAD (after k_wino4 on 12 waves and the k_emat rework): tools/profile_gpu.sh (kernel
# trace + stats, FETCH_SIZE, WRITE_SIZE, MFMA busy, matcher), then the kernel trace split by grid and queue
export TMPDIR=/tmp
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
bash tools/profile_gpu.sh || exit 1
python3 tools/r06/kernel_stats_by_grid.py gpurun_out/prof_trace --by-queue k_wino4 k_pnp k_tlm k_emat k_fmat k_ransac3d k_match > gpurun_out/prof_by_grid.csv && head -30 gpurun_out/prof_by_grid.csv
