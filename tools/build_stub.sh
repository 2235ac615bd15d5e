#!/bin/bash
# Host-floor library (vlib/stub.so): every source rebuilt with -DFDDM_STUB_KERNELS (csrc/common.h), so each launch is
# one empty kernel. Run with FDDM_HIP_LIB=$GRAFT_REPO_ROOT/vlib/stub.so; the results are garbage, the host
# enqueue time is the floor.
set -e
cd "$(dirname "$0")/../fddm-asr_amd"
mkdir -p ../vlib /tmp/stubo
objs=""
for f in csrc/*.hip; do
  stem=$(basename $f .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -fPIC -std=c++17 -w -DFDDM_STUB_KERNELS -c $f -o /tmp/stubo/$stem.o &
  objs="$objs /tmp/stubo/$stem.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../vlib/stub.so $objs
echo built vlib/stub.so
