#!/bin/bash
# Round-4 final validation and profiles at HEAD: GPU suite, smoke(), default bench line, then tools/profile_gpu.sh
export TMPDIR=/tmp
O=gpurun_out/r04final; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['roofline']['frac'], d['frontend_batch']['value'], d['monocular_hd']['value'], d['local_ba']['ms_per_call'])"
bash tools/profile_gpu.sh > $O/profile_gpu.log 2>&1 || { tail -20 $O/profile_gpu.log; exit 1; }
tail -8 $O/profile_gpu.log
echo done
