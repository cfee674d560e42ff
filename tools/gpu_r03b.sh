#!/bin/bash
# GPU session: the full -m gpu suite, then the matcher sweep (tools/match_sweep.sh).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
    -rA ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
[ -n "$SWEEP" ] && bash tools/match_sweep.sh
