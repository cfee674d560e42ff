#!/bin/bash
# Stall breakdown of the network kernels (tools/bench_net.py, 8 frames, 3 reps) for the Winograd
# (VS_WINO=1) and direct (VS_WINO=0) convs: two SQ counter passes each (MI355X_MICROARCH.md:
# WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES).  Output under gpurun_out/$TAG.
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
for w in 1 0; do
  for p in 1 2; do
    if [ $p = 1 ]; then C=$P1; else C=$P2; fi
    VS_WINO=$w timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/w${w}p$p -o pmc --output-format csv -- \
        python3 tools/bench_net.py --frames 8 --reps 3 > $O/w${w}p$p.log 2>&1 || exit 1
    echo "wino=$w pass $p ok"
  done
done
# HBM bytes of the Winograd kernels at 8 frames per launch (FETCH_SIZE / WRITE_SIZE in separate passes)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/$c -o pmc --output-format csv -- \
      python3 tools/bench_net.py --frames 8 --reps 3 > $O/$c.log 2>&1 || exit 1
  echo "$c ok"
done
