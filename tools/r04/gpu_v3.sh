#!/bin/bash
# matcher tail back to one chunk per pass (kernel VGPRs as before the tail change): parity, timing vs ab/tlm.so, final bench line
export TMPDIR=/tmp
O=gpurun_out/r04v3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_tracker.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for nl in old:ab/tlm.so head:visual-slam-pipeline_amd/libvslam_hip.so; do
  n=${nl%%:*}; lib=${nl#*:}
  VS_LIB_PATH=$lib timeout -k 10 120 python tools/bench_match.py --pairs 1,32,128 --reps 30 > $O/match_${n}_$r.jsonl 2>/dev/null || exit 1
  python3 -c "
import json
for l in open('$O/match_${n}_$r.jsonl'):
    if l.startswith('{'): d=json.loads(l); print('$n', $r, d['pairs'], d['us_per_launch'], d['mfma_frac'])"
done
done
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic_source'], d['match_roofline']['frontend_batch']['avg_launch_us'], d['frontend_batch']['value'], d['local_ba']['ms_per_call'], d['monocular_hd']['value'])"
echo done
