#!/bin/bash
# Timing-only library variants: rebuild one kernel source with extra -D flags and link it with the in-tree
# objects into vlib/<name>.so.   tools/build_variant.sh <name> <source stem> <flags...>
set -e
name=$1; stem=$2; shift 2
cd "$(dirname "$0")/../fddm-asr_amd"
mkdir -p ../vlib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -w "$@" -c csrc/$stem.hip -o /tmp/var_$stem_$name.o
objs=$(ls build/*.o | grep -v "build/$stem.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../vlib/$name.so $objs /tmp/var_$stem_$name.o
echo built vlib/$name.so
