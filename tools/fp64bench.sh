#!/bin/bash
# VALU issue price per instruction class on one MI355X (tools/fp64bench.hip): timings, then rocprofv3 passes
# with the cycle and issue counters.  Usage: bash tools/fp64bench.sh OUTDIR
# Summarise with: python3 tools/fp64bench_summary.py OUTDIR
set -u
out=${1:-gpurun_out/fp64bench}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 ./build/fp64bench 5 > "$out/times.jsonl" || { echo "fp64bench failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES \
    SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 --output-format csv -d "$out/pmc" -o p -- ./build/fp64bench 1 \
    > "$out/pmc.log" 2>&1 || { echo "pmc pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F64 \
    SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 --output-format csv -d "$out/pmc2" -o p -- \
    ./build/fp64bench 1 > "$out/pmc2.log" 2>&1 || { echo "pmc2 pass failed"; exit 1; }
echo "fp64bench ok"
