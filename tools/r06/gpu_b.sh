#!/bin/bash
# Round-6: the headline drive parity test + the default bench line (driver flags are now
# bench.py's defaults)
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06b}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline_drive.py -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed|processed|3d3d" $O/pytest.log | tail -8
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], d['warmup'], 'roofline', d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'net_mfma', d['network_mfma_tflops'])
print('upload', d['input_upload'])
print('fe', d['frontend_batch']['value'], 'mono', d['monocular_hd']['value'])"
