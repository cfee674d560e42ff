#!/bin/bash
# Round-6 final: CU sets spread over the eight XCDs (VS_SLAM_CU_SPREAD=1) vs contiguous ids, 3 rounds
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06spr}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py $H > $O/b_$tag.json 2> $O/b_$tag.err || { tail -20 $O/b_$tag.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']
print('$tag', d['value'], d['ms_per_step'], 'fmat', s.get('fmat_ransac'), 'match_spec', s.get('match_spec'), 'net', round(sum(v for k,v in s.items() if k.startswith('conv') or k.startswith('head')), 4))"
}
for r in 1 2 3; do
  run def$r VS_X=0
  run spr$r VS_SLAM_CU_SPREAD=1
done
