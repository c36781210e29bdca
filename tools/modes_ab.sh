#!/bin/bash
# A/B: for each kernel mode, time the default library and each named variant (tools/abl.sh per mode).
set -u
out=${OUT:-gpurun_out/mab}
for m in "se|" "sr|--method rk4" "pe|--mode pathline" "pr|--mode pathline --method rk4"; do
  n=${m%%|*}; a=${m#*|}
  BENCH_ARGS="$a" OUT=$out/$n bash tools/abl.sh base "$@" || exit 1
done
