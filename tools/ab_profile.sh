#!/bin/bash
# Same-box A/B of the bench's in-loop stage profiling (all / network / none), then one kernel trace of
# the tracker with no stage events (tracking-stream gaps between dependent kernels).
export TMPDIR=/tmp
O=gpurun_out/ab_prof
mkdir -p $O
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --track-profile-steps 0"
for r in 1 2 3; do
  for m in all network none; do
    timeout -k 10 300 python -u bench.py $ARGS --stage-profile $m > $O/${m}_$r.json 2> $O/${m}_$r.err || exit 1
    python3 -c "import json; d=json.loads([l for l in open('$O/${m}_$r.json') if l.startswith('{')][-1]); print('$m', $r, d['value'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o t --output-format csv -- python3 bench.py --steps 8 --warmup 2 \
    --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --track-profile-steps 0 --stage-profile none --render-workers 1 \
    > $O/trace.log 2>&1 && echo "trace ok"
