#!/bin/bash
# Network kernels only: parity tests of the network / extraction, then tools/bench_net.py with the
# direct kernels (VS_WINO=0) and the Winograd kernels, two rounds each (same box).  $TAG names the
# output directory.
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_monocular.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  VS_WINO=0 timeout -k 10 200 python -u tools/bench_net.py --tag direct > $O/net_direct_$r.json 2> $O/net_direct_$r.err || exit 1
  timeout -k 10 200 python -u tools/bench_net.py --tag wino > $O/net_wino_$r.json 2> $O/net_wino_$r.err || exit 1
done
python3 tools/net_summary.py $O
