#!/bin/bash
# Round-2 measurement of one bench workload: the bench line (with CPU baseline), the
# rocprofv3 kernel-trace stats of the same command, FETCH_SIZE / WRITE_SIZE passes merged
# into profiles/pmc_traffic.json (tools/make_traffic.py), the SQ/TA/TD counter passes, and
# the bench line again so that its roofline carries the measured traffic.
#   tools/profile_r02.sh OUTDIR KEY UNITS [bench args]
set -u
out=$1; key=$2; units=$3; shift 3
mkdir -p "$out" "$out/pmc"
export TMPDIR=/tmp
# the counter passes must see only the measured workload's kernels (bench.py's RK4 companion off)
export MOPS_BENCH_NO_RK4=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o p -- \
    python3 bench.py --no-cpu-baseline "$@" > "$out/stats.log" 2>&1 || { echo "stats failed"; exit 1; }
timeout -k 5 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex traj_kernel --output-format csv -d "$out/fetch" -o p -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > "$out/fetch.log" 2>&1 || { echo "fetch failed"; exit 1; }
timeout -k 5 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex traj_kernel --output-format csv -d "$out/write" -o p -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > "$out/write.log" 2>&1 || { echo "write failed"; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 5 240 rocprofv3 --pmc $grp --kernel-include-regex traj_kernel --output-format csv -d "$out/pmc/pass$i" -o p -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$out/pmc/pass$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py "$out/pmc" > "$out/pmc_summary.txt"
# after the counter passes: the record also carries their FP64 VALU work
python3 tools/make_traffic.py "$out" "$key" profiles/pmc_traffic.json "$units" "$out" > "$out/traffic.json" || { echo "traffic failed"; exit 1; }
cp profiles/pmc_traffic.json "$out/pmc_traffic.json"
timeout -k 10 400 python3 bench.py "$@" > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; exit 1; }
echo "profile ok"
