#!/bin/bash
# SQ counters of the tracker kernels (k_pnp_hyp: where a Jacobi round's ~1,400 cycles go), one PMC pass
export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
timeout -s KILL 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
want="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS"
have=""
for c in $want; do grep -qw "$c" $O/avail.txt && have="$have $c"; done
echo "counters:$have"
[ -n "$have" ] || exit 1
timeout -s KILL 300 rocprofv3 --pmc $have --kernel-trace -d $O/pmc -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0 --render-workers 1 > $O/pmc.log 2>&1 || exit 1
f=$(find $O/pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get('Kernel_Name', '')
    if not any(k in n for k in ('k_pnp_hyp', 'k_pnp_ransac', 'k_tlm_resolve', 'k_ba_chol')): continue
    key = n[:24]
    acc[key][r['Counter_Name']] += float(r['Counter_Value'])
    cnt[(key, r['Counter_Name'])] += 1
for k, d in acc.items():
    print(k, {c: round(v / max(1, cnt[(k, c)]), 1) for c, v in sorted(d.items())})
PY
echo done
