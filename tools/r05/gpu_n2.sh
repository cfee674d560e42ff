#!/bin/bash
# Round-5: NMS tile-round launches before k_nms_finish (4 = HEAD, 2, 1): post bench + parity
export TMPDIR=/tmp
O=gpurun_out/r05n2; mkdir -p $O
for v in r4 r1 r2; do
  if [ $v = r4 ]; then unset VS_LIB_PATH; else export VS_LIB_PATH=tools/r05/ab/libvslam_$v.so; fi
  for b in 8 32; do timeout -k 10 200 python -u tools/bench_post.py --batch $b --reps 40 > $O/post_${v}_$b.json 2> $O/post_${v}.err || { tail -5 $O/post_${v}.err; exit 1; }; done
  echo "$v B=8 $(cat $O/post_${v}_8.json | cut -c1-200)"
  echo "$v B=32 $(cat $O/post_${v}_32.json | cut -c1-200)"
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1; echo "$v pytest rc=$? $(tail -1 $O/pytest_$v.log)"
done
