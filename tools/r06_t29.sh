#!/bin/bash
# same-box A/B: conditioning kernels of this round (rows_mean on 64-column blocks, FiLM on register tiles, dW on 32x64
# tiles) vs the previous small.hip (abl/small_old.so)
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
ROUNDS=3 bash tools/ab.sh - "FDDM_HIP_LIB=$PWD/abl/small_old.so" > gpurun_out/r06_t29_ab.txt 2>&1 || exit 1
echo done
