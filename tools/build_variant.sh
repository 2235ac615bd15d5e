#!/bin/bash
# Timing-only library variants: rebuild one kernel source with extra -D flags and link it with the in-tree
# objects into abl/<name>.so (git-ignored; travels to the GPU box, FDDM_HIP_LIB=abl/<name>.so selects it).   tools/build_variant.sh <name> <source stem> <flags...>
set -e
name=$1; stem=$2; shift 2
cd "$(dirname "$0")/../fddm-asr_amd"
mkdir -p ../abl
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -w "$@" -c csrc/$stem.hip -o /tmp/var_$stem_$name.o
objs=$(ls build/*.o | grep -v "build/$stem.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../abl/$name.so $objs /tmp/var_$stem_$name.o
echo built abl/$name.so
