#!/bin/bash
# Round-6: next-but-one chain launched by the helper; tracker parity; bench A/B (speculation on/off, 16
# chain CUs); the reduced out-of-line repro of the EPnP divergence; host profile
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06g}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 tools/r06/epnp_b_repro > $O/epnp_b_repro.txt 2>&1; cat $O/epnp_b_repro.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline_drive.py tests/test_gpu_tracker_bench.py tests/test_gpu_tracker.py -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for cfg in "1 8" "0 8" "1 16" "1 8" "0 8" "1 16"; do
  set -- $cfg
  VS_SLAM_SPEC_TLM=$1 VS_SLAM_SPEC_CUS=$2 timeout -k 10 300 python -u bench.py $H > $O/bench_s$1_c$2.json 2> $O/bench_s$1_c$2.err || { tail -20 $O/bench_s$1_c$2.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_s$1_c$2.json').read().strip().splitlines()[-1])
print('spec_tlm=$1 spec_cus=$2', d['value'], d['ms_per_step'], 'conv1', d['roofline']['avg_launch_ms'])"
done
VS_SLAM_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py $H > $O/bench_hp.json 2> $O/bench_hp.err || { tail -20 $O/bench_hp.err; exit 1; }
grep "vs_slam" $O/bench_hp.err | head -24
