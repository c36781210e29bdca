#!/bin/bash
# FP64 VALU issue-rate calibration on one MI355X (tools/fp64bench.hip): timings, then one rocprofv3 pass
# with the cycle and instruction counters.  Usage: bash tools/fp64bench.sh OUTDIR
set -u
out=${1:-gpurun_out/fp64bench}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 ./build/fp64bench 5 > "$out/times.jsonl" || { echo "fp64bench failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 \
    SQ_INSTS_VALU_MUL_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d "$out/pmc" -o p -- ./build/fp64bench 1 \
    > "$out/pmc.log" 2>&1 || { echo "pmc pass failed"; exit 1; }
cat "$out/times.jsonl"
echo "fp64bench ok"
