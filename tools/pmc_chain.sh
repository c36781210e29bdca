#!/bin/bash
# FETCH/WRITE PMC passes for the configs 4/5 trajectory launches (one 30-day chain reduced to
# 2 daily pairs for config 4; the first monthly pair for config 5), merged into
# profiles/pmc_traffic.json under bench.py's workload keys, then the two bench lines re-run so
# that their roofline.traffic is filled.  One device, one call; outputs under $1.
set -u
out=${1:-gpurun_out/pmcc}
mkdir -p "$out"
export TMPDIR=/tmp
# the counter passes must see only the measured workload's kernels (bench.py's RK4 companion off)
export MOPS_BENCH_NO_RK4=1
for c in "4:--pairs 2:orrs18to6_chain4_euler_10000000_seg720" "5:--pairs 1:orrs18to6_chain5_euler_12500000_seg4320"; do
  n=${c%%:*}; r=${c#*:}; a=${r%%:*}; key=${r#*:}
  timeout -k 5 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex traj_kernel --output-format csv -d "$out/c$n/fetch" -o p -- \
      python3 bench.py --config $n $a --steps 1 --warmup 0 --no-cpu-baseline > "$out/c$n.fetch.log" 2>&1 || { echo "c$n fetch failed"; exit 1; }
  timeout -k 5 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex traj_kernel --output-format csv -d "$out/c$n/write" -o p -- \
      python3 bench.py --config $n $a --steps 1 --warmup 0 --no-cpu-baseline > "$out/c$n.write.log" 2>&1 || { echo "c$n write failed"; exit 1; }
  python3 tools/make_traffic.py "$out/c$n" "$key" profiles/pmc_traffic.json || exit 1
done
cp profiles/pmc_traffic.json "$out/pmc_traffic.json"
timeout -k 10 400 python3 bench.py --config 4 --steps 1 --warmup 0 > "$out/c4.json" 2> "$out/c4.err" || { echo "c4 failed"; exit 1; }
timeout -k 10 400 python3 bench.py --config 5 --steps 1 --warmup 0 > "$out/c5.json" 2> "$out/c5.err" || { echo "c5 failed"; exit 1; }
echo "pmc chain ok"
