#!/bin/bash
# fwd8 fine stamps: chunk ends of the 5th (half-0 alpha) and 6th (half-0 beta) phase call of every workgroup
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
for n in 5 6; do
  A8_FINE=$n FDDM_HIP_LIB=$PWD/abl/fine$n.so timeout -k 10 120 python -u tools/probe/a8_stamps.py > gpurun_out/r06_t22_fine$n.log 2>&1 || exit 1
done
echo done
