#!/bin/bash
# Winograd F(2x2, 3x3) convs: network parity tests (torch fp64 / oracle CPU network tolerance, all
# geometries, extraction end to end), then the network alone (tools/bench_net.py) with the direct
# kernels (VS_WINO=0) and Winograd, then the headline bench both ways.
mkdir -p gpurun_out/r03l
export TMPDIR=/tmp
O=gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_monocular.py tests/test_gpu_onnx.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  VS_WINO=0 timeout -k 10 200 python -u tools/bench_net.py --tag direct > $O/net_direct_$r.json 2> $O/net_direct_$r.err || exit 1
  timeout -k 10 200 python -u tools/bench_net.py --tag wino > $O/net_wino_$r.json 2> $O/net_wino_$r.err || exit 1
done
python3 - <<'PY'
import json
for t in ("direct", "wino"):
    d = json.loads(open(f"gpurun_out/r03l/net_{t}_2.json").read().strip().splitlines()[-1])
    for k, v in d.items():
        if k.startswith("frames"):
            print(t, k, v.get("network_ms_per_launch"), {kk: (vv.get("ms_per_launch"), vv.get("frac")) for kk, vv in v.items() if isinstance(vv, dict)})
PY
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --track-profile-steps 0"
for r in 1 2; do
  for v in "D|VS_WINO=0" "W|VS_WINO=1" "W40|VS_WINO=1,VS_SLAM_TRACK_CUS=40" "W48|VS_WINO=1,VS_SLAM_TRACK_CUS=48"; do
    name=${v%%|*}; envs=${v#*|}; envs=${envs//,/ }
    env $envs timeout -k 10 300 python -u bench.py $ARGS > $O/${name}_$r.json 2> $O/${name}_$r.err || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$O/${name}_$r.json') if l.startswith('{')][-1]); print('$name', $r, d['value'], d['roofline']['frac'], d['network_tflops'])"
  done
done
