#!/bin/bash
# A/B timing on one GPU box: the headline tracker bench alternated between library builds and
# environment settings (box-to-box variance is several percent, so comparisons stay on one box).
# Each variant: "name|env assignments" in $VARIANTS (';'-separated), $ROUNDS alternations.
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
: "${ROUNDS:=3}"
: "${VARIANTS:=A|VS_LIB_PATH=ab/libA.so;B|VS_LIB_PATH=ab/libB.so}"
IFS=';' read -ra VS <<< "$VARIANTS"
for r in $(seq 1 $ROUNDS); do
  for v in "${VS[@]}"; do
    name=${v%%|*}; envs=${v#*|}
    env $envs timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-frontend \
        --mono-steps 0 > $O/${name}_$r.json 2> $O/${name}_$r.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/${name}_$r.json')); print('$name', $r, d['value'], d['ms_per_step'])"
  done
done
