#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_monocular.py tests/test_gpu_midas.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=r04d ROUNDS=2 LIBS="base:ab/base.so ws0:ab/ws0.so ws1:ab/ws1.so ws2:ab/ws2.so" bash tools/r04/net_ab.sh || exit 1
echo done
