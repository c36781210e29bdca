#!/bin/bash
# The memory-return counters per engine variant ("base" = the product library), bench.py ${BENCH_ARGS}:
# TD busy cycles, GRBM active cycles, vector-L1 (TCP) tag accesses (64 B each, tools/membench.hip) and
# L1 -> L2 read requests (128 B each), per traj_kernel dispatch.
#   OUT=gpurun_out/x BENCH_ARGS="--config 3 --pairs 1" bash tools/pmc_td.sh base nocoop ...
set -u
out=${OUT:-gpurun_out/pmctd}
mkdir -p $out
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L=$PWD/build/variants/libmops_$v.so; fi
  MOPS_TRAJ_LIB=$L timeout -s KILL 150 rocprofv3 --pmc TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum \
      TCP_TCC_READ_REQ_sum --kernel-include-regex traj_kernel \
      --output-format csv -d $out/$v -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} \
      > $out/$v.log 2>&1 || { echo "$v failed"; tail -5 $out/$v.log; exit 1; }
  python3 - $out/$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
tot = collections.Counter(); n = collections.Counter()
for r in csv.DictReader(open(f)):
    tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
d = n["GRBM_GUI_ACTIVE"]
busy = tot["TD_TD_BUSY_sum"] / 256 / (tot["GRBM_GUI_ACTIVE"] / 8)
print(sys.argv[1].split("/")[-1], "dispatches", d, "TD busy %.3f" % busy,
      "L1 accesses/dispatch %.4g (x64 B)" % (tot["TCP_TOTAL_CACHE_ACCESSES_sum"] / d),
      "L1->L2 req/dispatch %.4g (x128 B)" % (tot["TCP_TCC_READ_REQ_sum"] / d),
      "GRBM cycles/dispatch %.4g" % (tot["GRBM_GUI_ACTIVE"] / d / 8))
PY
done
