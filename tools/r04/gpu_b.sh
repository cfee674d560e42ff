#!/bin/bash
# New parity tests (large independent goldens, ONNX desc tails) + bench feature dump.
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_golden.py tests/test_gpu_onnx.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dump_bench_features.py $O/bench_features.npz || exit 1
echo done
