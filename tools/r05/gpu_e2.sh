#!/bin/bash
# Round-5: k_emat with 8 waves x 4 solves per round (vs 4 x 8): A/B + emat parity
export TMPDIR=/tmp
O=gpurun_out/r05e2; mkdir -p $O
VS_LIB_PATH=tools/r05/ab/libvslam_old.so timeout -k 10 120 python -u tools/r05/bench_emat.py > $O/old.jsonl 2> $O/old.err || { tail -5 $O/old.err; exit 1; }
timeout -k 10 120 python -u tools/r05/bench_emat.py > $O/new.jsonl 2> $O/new.err || { tail -5 $O/new.err; exit 1; }
echo old; cat $O/old.jsonl; echo new; cat $O/new.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_emat.py tests/test_golden.py tests/test_gpu_monocular.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed" $O/pytest.log | tail -3
