#!/bin/bash
# Same-box A/B of the network kernels: bit-identity of the network outputs between two library
# builds, then tools/bench_net.py alternated (ROUNDS rounds).  A = ab/base.so, B = the in-tree build.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-netab}; mkdir -p $O
: "${ROUNDS:=3}"
for v in A B; do
  lib=ab/base.so; [ $v = B ] && lib=visual-slam-pipeline_amd/libvslam_hip.so
  VS_LIB_PATH=$lib timeout -k 10 120 python -u tools/net_dump.py $O/out_$v.npz || exit 1
done
python3 - <<PY || exit 1
import numpy as np
a, b = np.load("$O/out_A.npz"), np.load("$O/out_B.npz")
for k in a.files:
    same = np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))
    print(k, "bit-identical" if same else f"DIFFERS max|d| {np.abs(a[k]-b[k]).max():.3e}")
PY
for r in $(seq 1 $ROUNDS); do
  for v in A B; do
    lib=ab/base.so; [ $v = B ] && lib=visual-slam-pipeline_amd/libvslam_hip.so
    VS_LIB_PATH=$lib timeout -k 10 200 python -u tools/bench_net.py --tag $v > $O/net_${v}_$r.json 2> $O/net_${v}_$r.err || exit 1
    python3 -c "
import json; d=json.loads(open('$O/net_${v}_$r.json').read().strip().splitlines()[-1])
for k in ('frames_8','frames_32'):
    L=d[k]['layers']; print('$v', $r, k, d[k]['network_ms_per_launch'], {n: L[n]['ms_per_launch'] for n in ('conv1_fused','conv2a','conv2b_pool','conv3a','conv3b_pool','conv4a','head_a','head_b') if n in L})"
  done
done
