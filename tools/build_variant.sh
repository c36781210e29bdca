#!/bin/bash
# Build build/variants/libmops_<name>.so with extra -D flags (perf experiments;
# time them with tools/occupancy_sweep.sh <name>...).
set -eu
name=$1; shift
cd "$(dirname "$0")/.."
mkdir -p build/variants
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Iinclude "$@" \
    -o build/variants/libmops_$name.so mops_amd/csrc/mops_engine.hip mops_amd/csrc/mops_api.cpp \
    mops_amd/csrc/mops_io.cpp mops_amd/csrc/mops_netcdf.cpp
echo "built $name"
