#!/bin/bash
# Round-6: SQ stall breakdown of k_wino4 (network alone, 8 frames): two counter passes
export TMPDIR=/tmp
O=gpurun_out/${GPU_OUT:-r06j}; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
for p in 1 2; do
  if [ $p = 1 ]; then C=$P1; else C=$P2; fi
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/w1p$p -o pmc --output-format csv -- \
      python3 tools/bench_net.py --frames 8 --reps 3 > $O/w1p$p.log 2>&1 || exit 1
  echo "pass $p ok"
done
python3 tools/pmc_breakdown.py $O 2>&1 | head -20
