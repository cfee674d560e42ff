#!/bin/bash
# Tracker bottleneck view over $VARIANTS (name|env, ',' between assignments): headline bench with the
# host profile (VS_SLAM_HOST_PROFILE=1), one round each, then a kernel trace of variant $TRACE_ENV.
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
O=gpurun_out/$TAG
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --track-profile-steps 0"
for v in $VARIANTS; do
  name=${v%%|*}; envs=${v#*|}; envs=${envs//,/ }
  env VS_SLAM_HOST_PROFILE=1 $envs timeout -k 10 300 python -u bench.py $ARGS > $O/${name}.json 2> $O/${name}.err || exit 1
  python3 -c "import json; d=json.loads([l for l in open('$O/${name}.json') if l.startswith('{')][-1]); print('$name', d['value'], d['network_tflops'])"
  grep -E "process_frame|extract wait|track_local_map: sync|phase" $O/${name}.err | head -9
done
if [ -n "$TRACE_ENV" ]; then
  env ${TRACE_ENV//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 \
      --render-workers 1 > $O/trace.log 2>&1 || exit 1
  python3 tools/trace_tracker.py $O/trace/trace_kernel_trace.csv | head -14
fi
