#!/bin/bash
# same-box A/B: default vs fwd7 forward everywhere vs encoder CU caps one step up
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
ROUNDS=2 bash tools/ab.sh - "FDDM_ATTN_KERNELS=fwd7" "FDDM_ENC_CUS=208" "FDDM_ENC_CUS_CONV=144" > gpurun_out/r06_t18_ab.txt 2>&1 || exit 1
echo done
