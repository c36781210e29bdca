#!/bin/bash
# Build round-3 kernel variants (MAXV 7 only) into build/variants/ (CPU side).
set -eu
cd "$(dirname "$0")/.."
rm -f build/variants/*.so
tools/build_variant.sh base7 -DMOPS_ONLY7 &
tools/build_variant.sh trig1 -DMOPS_ONLY7 -DMOPS_TRIG_ONESIDED=1 &
tools/build_variant.sh div1 -DMOPS_ONLY7 -DMOPS_DIV3_ONESIDED=1 &
tools/build_variant.sh both1 -DMOPS_ONLY7 -DMOPS_TRIG_ONESIDED=1 -DMOPS_DIV3_ONESIDED=1 &
wait
