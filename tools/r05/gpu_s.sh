#!/bin/bash
# Round-5: post-processing fusion (decode inside the local-maximum pass, XCD-aware tiles, the
# descriptor grid normalised at the sampled corners): smoke, parity, the post bench, PMC bytes
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spcf.py tests/test_gpu_tracker.py tests/test_gpu_tracker_bench.py tests/test_gpu_batch.py tests/test_gpu_onnx.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/bench_post.py --batch 32 --reps 20 > $O/post.json 2> $O/post.err || { tail -5 $O/post.err; exit 1; }
cat $O/post.json
PMC_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --render-workers 1 --ba-reps 0"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/prof_fetch -o fetch --output-format csv -- \
    python3 bench.py $PMC_ARGS > $O/prof_fetch.log 2>&1 && echo "fetch ok" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/prof_write -o write --output-format csv -- \
    python3 bench.py $PMC_ARGS > $O/prof_write.log 2>&1 && echo "write ok"
