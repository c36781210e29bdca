#!/bin/bash
# Level-pair record build tile variants (MAXV 7 only) into build/variants/.
set -eu
cd "$(dirname "$0")/.."
tools/build_variant.sh rec64x16 -DMOPS_ONLY7 &
tools/build_variant.sh rec32x16 -DMOPS_ONLY7 -DMOPS_REC_TV=32 -DMOPS_REC_TK=16 &
tools/build_variant.sh rec32x32 -DMOPS_ONLY7 -DMOPS_REC_TV=32 -DMOPS_REC_TK=32 &
tools/build_variant.sh rec64x8 -DMOPS_ONLY7 -DMOPS_REC_TV=64 -DMOPS_REC_TK=8 &
wait
