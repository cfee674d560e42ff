#!/bin/bash
# rocprofv3 passes over bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats (per-kernel durations; the summary committed under profiles/)
#   2. FETCH_SIZE and 3. WRITE_SIZE in separate PMC passes (TCC slots; MI355X_MICROARCH.md)
# Each pass has its own time limit and the chain stops at the first failure.
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out
# Single-size passes: --no-frontend --mono-steps 0 leaves only the tracker, whose network launches are
# all one extraction chunk (8 frames), so per-launch durations and bytes divide by one frame count.
ARGS=${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --render-workers 1}
PMC_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --render-workers 1"
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_trace -o trace --output-format csv -- \
    python3 $R/bench.py $ARGS > $OUT/prof_trace.log 2>&1 && echo "trace ok" &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/prof_fetch -o fetch --output-format csv -- \
    python3 $R/bench.py $PMC_ARGS --ba-reps 0 > $OUT/prof_fetch.log 2>&1 && echo "fetch ok" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/prof_write -o write --output-format csv -- \
    python3 $R/bench.py $PMC_ARGS --ba-reps 0 > $OUT/prof_write.log 2>&1 && echo "write ok"
# 4. matrix-core busy cycles of every kernel in the bench (conv1 is the roofline kernel), and
# 5./6. the matcher alone (tools/bench_match.py at 32 and 512 pairs per launch): kernel trace, then
# the same MFMA counters.  MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
# GRBM_GUI_ACTIVE / 8), summarised by tools/summarize_profiles.py.
[ -z "$SKIP_MFMA" ] &&
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/prof_mfma \
    -o mfma --output-format csv -- python3 $R/bench.py $PMC_ARGS --ba-reps 0 > $OUT/prof_mfma.log 2>&1 &&
echo "mfma ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_match -o match --output-format csv -- \
    python3 $R/tools/bench_match.py --pairs 1,32,512 --reps 20 > $OUT/prof_match.log 2>&1 && echo "match trace ok" &&
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/prof_match_mfma \
    -o match_mfma --output-format csv -- python3 $R/tools/bench_match.py --pairs 32,512 --reps 5 \
    > $OUT/prof_match_mfma.log 2>&1 && echo "match mfma ok"
