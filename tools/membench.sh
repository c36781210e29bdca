#!/bin/bash
# Memory-path calibration on one MI355X (tools/membench.hip): timings, then one rocprofv3 pass per
# counter group (FETCH_SIZE; TD busy + TD->SP sends + GRBM; TCP accesses + L1->L2 requests).
# Usage: bash tools/membench.sh OUTDIR
set -u
out=${1:-gpurun_out/membench}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 120 ./build/membench 3 > "$out/times.jsonl" || { echo "membench failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o p -- ./build/membench 1 > "$out/fetch.log" 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TD_TD_BUSY_sum TD_TD_SP_TRAFFIC_sum GRBM_GUI_ACTIVE --output-format csv -d "$out/td" -o p -- ./build/membench 1 > "$out/td.log" 2>&1 || { echo "td pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$out/tcp" -o p -- ./build/membench 1 > "$out/tcp.log" 2>&1 || { echo "tcp pass failed"; exit 1; }
echo "membench ok"
