#!/bin/bash
# Build the round-3 kernel variants (MAXV 7 only) into build/variants/ (CPU side).
set -eu
cd "$(dirname "$0")/.."
tools/build_variant.sh base7 -DMOPS_ONLY7 &
tools/build_variant.sh hexpairs -DMOPS_ONLY7 -DMOPS_HEX_PAIRS=1 &
tools/build_variant.sh sqrt1 -DMOPS_ONLY7 -DMOPS_SQRT_ONESIDED=1 &
wait
