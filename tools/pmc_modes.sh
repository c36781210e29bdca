#!/bin/bash
# PMC passes (instruction mix, waits, TA/TD busy) for streamline-Euler and
# pathline-Euler traj_kernel launches; summaries in $1/<mode>.txt.
set -u
out=${1:-gpurun_out/pmc}
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
G2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
for mode in se pe; do
  case $mode in se) A="";; pe) A="--mode pathline";; esac
  BENCH_ARGS="$A" bash tools/pmc.sh "$out/$mode" "$G1" "$G2" || exit 1
  python3 tools/pmc_summary.py "$out/$mode" > "$out/$mode.txt"
done
echo pmc-modes ok
