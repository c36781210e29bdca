#!/bin/bash
# Instruction mix of traj_kernel for one bench call (two SQ counter passes, 8 counters each):
#   tools/pmc_mix.sh OUTDIR [bench args]   -> OUTDIR/mix.txt (per-dispatch means, per wave-step)
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
# the counter passes must see only the measured workload's kernels (bench.py's RK4 companion off)
export MOPS_BENCH_NO_RK4=1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64" \
           "SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex traj_kernel --output-format csv -d "$out/pass$i" -o p -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$out/pass$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py "$out" > "$out/mix.txt" && cat "$out/mix.txt"
