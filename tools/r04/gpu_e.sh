#!/bin/bash
# network A/B (base / interleaved / interleaved + setprio), MiDaS alone A/B, headline bench A/B
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
TAG=r04e ROUNDS=2 LIBS="base:ab/base.so ws1:ab/ws1.so wp1:ab/wp1.so" bash tools/r04/net_ab.sh || exit 1
for r in 1 2; do
  for nl in base:ab/base.so head:visual-slam-pipeline_amd/libvslam_hip.so; do
    n=${nl%%:*}; lib=${nl#*:}
    VS_LIB_PATH=$lib timeout -k 10 120 python -u tools/bench_midas.py > $O/midas_${n}_$r.json 2>&1 || exit 1
    echo "midas $n $r $(tail -1 $O/midas_${n}_$r.json | cut -c1-200)"
  done
done
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for r in 1 2; do
  for nl in base:ab/base.so head:visual-slam-pipeline_amd/libvslam_hip.so; do
    n=${nl%%:*}; lib=${nl#*:}
    VS_LIB_PATH=$lib timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${n}_$r.json').read().strip().splitlines()[-1]); print('bench $n $r', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['network_tflops'])"
  done
done
echo done
