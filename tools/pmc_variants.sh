#!/bin/bash
# One SQ counter pass per engine variant ("base" = the product library), bench.py ${BENCH_ARGS} (default config 2):
#   OUT=gpurun_out/x bash tools/pmc_variants.sh base nopair ...
set -u
out=${OUT:-gpurun_out/pmcv}
mkdir -p $out
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L=$PWD/build/variants/libmops_$v.so; fi
  MOPS_TRAJ_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-include-regex traj_kernel \
      --output-format csv -d $out/$v -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} \
      > $out/$v.log 2>&1 || { echo "$v failed"; tail -5 $out/$v.log; exit 1; }
  python3 - $out/$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
tot = collections.Counter()
for r in csv.DictReader(open(f)):
    tot[r["Counter_Name"]] += float(r["Counter_Value"])
w = tot["SQ_WAVES"]
print(sys.argv[1].split("/")[-1], {k: round(v / w, 1) for k, v in sorted(tot.items()) if k != "SQ_WAVES"}, "waves", int(w))
PY
done
