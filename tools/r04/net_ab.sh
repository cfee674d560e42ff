#!/bin/bash
# Same-box A/B of network kernel builds: bit-identity of the network outputs against the first
# library, then tools/bench_net.py alternated over the libraries (ROUNDS rounds).
# LIBS="name:path name:path ..." (default: base = ab/base.so, head = the in-tree build)
export TMPDIR=/tmp
O=gpurun_out/${TAG:-netab}; mkdir -p $O
: "${ROUNDS:=3}"
: "${LIBS:=base:ab/base.so head:visual-slam-pipeline_amd/libvslam_hip.so}"
first=""
for nl in $LIBS; do
  n=${nl%%:*}; lib=${nl#*:}
  VS_LIB_PATH=$lib timeout -k 10 120 python -u tools/net_dump.py $O/out_$n.npz || exit 1
  [ -z "$first" ] && first=$n
  python3 - <<PY || exit 1
import numpy as np
a, b = np.load("$O/out_$first.npz"), np.load("$O/out_$n.npz")
for k in a.files:
    same = np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))
    print("$n vs $first", k, "bit-identical" if same else f"DIFFERS max|d| {np.abs(a[k]-b[k]).max():.3e}")
PY
done
rm -f $O/out_*.npz  # 25 MB each: keep gpurun_out under the 64 MiB copy-back limit
for r in $(seq 1 $ROUNDS); do
  for nl in $LIBS; do
    n=${nl%%:*}; lib=${nl#*:}
    VS_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_net.py --tag $n > $O/net_${n}_$r.json 2> $O/net_${n}_$r.err || exit 1
    python3 -c "
import json; d=json.loads(open('$O/net_${n}_$r.json').read().strip().splitlines()[-1])
for k in ('frames_8','frames_32'):
    L=d[k]['layers']; print('$n', $r, k, d[k]['network_ms_per_launch'], {n: L[n]['ms_per_launch'] for n in ('conv1_fused','conv2a','conv2b_pool','conv3a','conv3b_pool','conv4a','head_a','head_b') if n in L})"
  done
done
