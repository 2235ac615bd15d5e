#!/bin/bash
# WavLM attention forward: register target 2 (base, 156 VGPRs = 3 waves / SIMD) vs 4 (128 VGPRs, spills)
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
for v in base f5w4 base f5w4; do
  if [ $v = base ]; then unset FDDM_HIP_LIB; else export FDDM_HIP_LIB=$PWD/abl/$v.so; fi
  echo "== $v" >> gpurun_out/r06_t35.txt
  timeout -k 10 120 python -u tools/wavlm_attn_time.py >> gpurun_out/r06_t35.txt 2>&1 || exit 1
done
echo done
