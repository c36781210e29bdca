#!/bin/bash
# Issue-pipe occupancy of the trajectory kernel (one PMC pass, SQ block only + GRBM):
# SQ_ACTIVE_INST_{VALU,SCA,VMEM,LDS,ANY} count quad-cycles in which a wave of a SIMD issued that
# kind of instruction, SQ_BUSY_CYCLES the SQ's busy cycles; per-SIMD fractions are taken against
# GRBM_GUI_ACTIVE x SIMDs (tools/make_traffic.py, "issue" block).
set -u
out=${1:-gpurun_out/issue}
mkdir -p "$out"
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS \
    SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex traj_kernel \
    --output-format csv -d "$out/issue" -o p -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:-} > "$out/issue.log" 2>&1 || { echo "issue pass failed"; exit 1; }
echo "issue ok"
