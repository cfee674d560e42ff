#!/bin/bash
# Headline bench (tracker only, 40 steps) over $VARIANTS (space-separated name|env, ',' between
# assignments), $ROUNDS rounds on one box; $TAG names the output directory.
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --track-profile-steps 0"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    name=${v%%|*}; envs=${v#*|}; envs=${envs//,/ }
    env $envs timeout -k 10 300 python -u bench.py $ARGS > $O/${name}_$r.json 2> $O/${name}_$r.err || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$O/${name}_$r.json') if l.startswith('{')][-1]); print('$name', $r, d['value'], d['roofline']['frac'], d['network_tflops'])"
  done
done
