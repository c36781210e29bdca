#!/bin/bash
# Round-3 measurement of bench workloads: for each "tag|key|units|bench args" the rocprofv3 kernel
# stats, the FETCH_SIZE / WRITE_SIZE passes merged into profiles/pmc_traffic.json
# (tools/make_traffic.py), the SQ/TA/TD counter passes (tools/profile_r02.sh), and the bench line.
#   tools/profile_r03.sh OUTDIR "c2|ec30to60_streamline_euler_1000000_seg720_p2c6|1|" ...
set -u
out=$1; shift
mkdir -p "$out"
for spec in "$@"; do
  IFS='|' read -r tag key units args <<< "$spec"
  t0=$(date +%s)
  bash tools/profile_r02.sh "$out/$tag" "$key" "$units" $args > "$out/$tag.log" 2>&1
  rc=$?
  echo "$tag rc=$rc $(( $(date +%s) - t0 ))s"
  [ $rc -ne 0 ] && { tail -5 "$out/$tag.log"; exit $rc; }
done
exit 0
