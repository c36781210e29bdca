#!/bin/bash
# One GPU call: run each "name|command" step under its own time limit, write
# output to $OUT/<name>.log, continue past ordinary failures (rc 1/2), and stop
# after a crash or a time limit (124/134/137/139) so nothing else touches the GPU.
set -u
OUT=${OUT:-gpurun_out/r2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%|*}; cmd=${step#*|}
  t0=$(date +%s)
  bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "step $name rc=$rc $(( $(date +%s) - t0 ))s"
  case $rc in 124|134|137|139) echo "stopping after $name"; exit $rc;; esac
done
