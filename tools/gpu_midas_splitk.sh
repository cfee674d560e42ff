#!/bin/bash
# MiDaS kernel A/B: MiDaS + monocular parity tests, then MiDaS alone (tools/bench_midas.py) over
# $VARIANTS (space-separated name|env assignments, ',' between assignments; default: split-K off / on)
# on the same box, and a kernel trace of the default build.
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
VARIANTS=${VARIANTS:-"nosplit|VS_MIDAS_SPLITK_WGS=0 default|VS_NONE=1"}
timeout -k 10 600 python -u -m pytest tests/test_gpu_midas.py tests/test_gpu_monocular.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in $VARIANTS; do
    name=${v%%|*}; envs=${v#*|}; envs=${envs//,/ }
    env $envs timeout -k 10 200 python -u tools/bench_midas.py > $O/midas_${name}_$r.json 2> $O/midas_${name}_$r.err || exit 1
    echo "$name $r $(tail -1 $O/midas_${name}_$r.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o midas --output-format csv -- \
    python3 tools/bench_midas.py --reps 5 > $O/prof.log 2>&1 || exit 1
echo prof ok
