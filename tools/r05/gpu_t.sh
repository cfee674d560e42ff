#!/bin/bash
# Round-5: the staged decode in k_nms_lmax: smoke, post parity, the post bench
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tracker_bench.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do timeout -k 10 300 python -u tools/bench_post.py --batch 32 --reps 20 || exit 1; done > $O/post.json 2> $O/post.err
cat $O/post.json
for i in 1 2; do timeout -k 10 300 python -u tools/bench_post.py --batch 8 --reps 40 || exit 1; done > $O/post8.json 2>> $O/post.err
cat $O/post8.json
