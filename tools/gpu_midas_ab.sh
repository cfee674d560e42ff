#!/bin/bash
# MiDaS stride-1 3x3 convs on the Winograd kernel: MiDaS / network / monocular parity tests, then the
# config[4] monocular stream (bench.py monocular_hd block) with VS_WINO=0 / 1 on the same box.
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_midas.py tests/test_gpu_parity.py tests/test_gpu_monocular.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-frontend --mono-steps 6 --ba-reps 0 --track-profile-steps 0"
for r in 1 2; do
  for w in 0 1; do
    VS_WINO=$w timeout -k 10 300 python -u bench.py $ARGS > $O/mono_w${w}_$r.json 2> $O/mono_w${w}_$r.err || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$O/mono_w${w}_$r.json') if l.startswith('{')][-1]); m=d['monocular_hd']; print('wino=$w', $r, d['value'], m['value'], m['midas']['stage_ms_per_frame'], m['midas']['roofline']['frac'])"
  done
done
