#!/bin/bash
# Full measurement for the round: bench (with CPU baseline), rocprofv3 kernel
# stats of the same command, and FETCH/WRITE PMC passes for the roofline traffic.
set -u
out=${1:-gpurun_out/round}
mkdir -p "$out"
export TMPDIR=/tmp
# the box whose cycles the PMC entry carries (bench.py prints it beside its own): host name + GPU uuid / PCI address
python3 -c "import bench; print(bench.bench_host())" > "$out/host.txt"
# the counter passes must see only the measured workload's kernels (bench.py's RK4 companion off)
export MOPS_BENCH_NO_RK4=1
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o p -- \
    python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$out/stats.log" 2>&1 || { echo "stats failed"; exit 1; }
timeout -k 5 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex traj_kernel --output-format csv -d "$out/fetch" -o p -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:-} > "$out/fetch.log" 2>&1 || { echo "fetch failed"; exit 1; }
timeout -k 5 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex traj_kernel --output-format csv -d "$out/write" -o p -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:-} > "$out/write.log" 2>&1 || { echo "write failed"; exit 1; }
timeout -k 5 300 rocprofv3 --pmc TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum \
    --kernel-include-regex traj_kernel --output-format csv -d "$out/td" -o p -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:-} > "$out/td.log" 2>&1 || { echo "td failed"; exit 1; }
timeout -k 5 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex traj_kernel --output-format csv -d "$out/pmc" -o p -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:-} > "$out/pmc.log" 2>&1 || { echo "pmc failed"; exit 1; }
timeout -k 5 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS \
    SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex traj_kernel --output-format csv \
    -d "$out/issue" -o p -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:-} > "$out/issue.log" 2>&1 \
    || { echo "issue failed"; exit 1; }
timeout -k 5 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 \
    SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 --kernel-include-regex traj_kernel --output-format csv \
    -d "$out/mix" -o p -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:-} > "$out/mix.log" 2>&1 \
    || { echo "mix failed"; exit 1; }
# then: tools/make_traffic.py $out KEY profiles/pmc_traffic.json UNITS && tools/merge_issue.py $out/issue KEY profiles/pmc_traffic.json
echo "profile ok"
