#!/bin/bash
# Round-5: GPU suite + default bench line after F(4x4,3x3)
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['frontend_batch']['value'], d['monocular_hd']['value'], d['local_ba']['ms_per_call'])"
tail -30 $O/bench.err
echo done
