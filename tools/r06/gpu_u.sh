#!/bin/bash
# Round-6: kernel trace of the config[4] monocular block (k_emat's share of its steps)
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/mono -o mono --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-frontend --steps 1 --warmup 1 --ba-reps 0 --render-workers 1 > $O/mono.json 2> $O/mono.err || { tail -5 $O/mono.err; exit 1; }
python3 tools/r06/kernel_stats_by_grid.py $O/mono k_emat k_wino4 k_mid k_match k_fmat > $O/mono_by_grid.csv
python3 -c "
import json; d=json.loads(open('$O/mono.json').read().strip().splitlines()[-1]); m=d['monocular_hd']
print('mono', m['value'], m['ms_per_step'], m['steps'])"
head -12 $O/mono_by_grid.csv
