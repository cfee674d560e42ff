#!/bin/bash
# Round-6: k_wino4 with the padded LDS patch (conflict-free transform reads): network parity, network alone,
# LDS conflict PMC pass, headline A/B against the previous library (git HEAD build in gpurun_out/oldlib)
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06r}; mkdir -p $O
( while sleep 45; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "network or extract" > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -12
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_net.py --frames 8,32 --reps 10 > $O/net_new.json 2> $O/net_new.err || { tail $O/net_new.err; exit 1; }
VS_LIB_PATH=$PWD/tools/r06/oldlib/libvslam_hip.so timeout -k 10 300 python -u tools/bench_net.py --frames 8,32 --reps 10 > $O/net_old.json 2> $O/net_old.err || { tail $O/net_old.err; exit 1; }
python3 - <<PY
import json
for t in ("new", "old"):
    for l in open("$O/net_%s.json" % t):
        try: d = json.loads(l)
        except Exception: continue
        print(t, json.dumps(d)[:400])
PY
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-trace -d $O/pmc -o pmc --output-format csv -- python3 tools/bench_net.py --frames 8 --reps 3 > $O/pmc.log 2>&1 && python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob("$O/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]; acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:5]:
    print(k, "lds_conflict %.3f" % (d.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, d.get("SQ_LDS_IDX_ACTIVE", 1))),
          "wait_lds %.3f" % (d.get("SQ_WAIT_INST_LDS", 0) / max(1, d.get("SQ_WAVE_CYCLES", 1))))
PY
H="--no-cpu-baseline --no-frontend --mono-steps 0 --ba-reps 0"
for t in new old new old; do
  L=""; [ $t = old ] && L=$PWD/tools/r06/oldlib/libvslam_hip.so
  VS_LIB_PATH=$L timeout -k 10 300 python -u bench.py $H > $O/b_$t.json 2> $O/b_$t.err || { tail -20 $O/b_$t.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]); s=d['stage_ms_per_frame']
net=sum(v for k,v in s.items() if k.startswith('conv') or k.startswith('head') or k=='gray_norm')
print('$t', d['value'], d['ms_per_step'], 'net/frame %.4f' % net, 'conv1', d['roofline']['avg_launch_ms'])"
done
