#!/bin/bash
# fused KL occupancy variants: 4 / 5 waves per SIMD register targets
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
for v in base klw4 klw5 base; do
  if [ $v = base ]; then unset FDDM_HIP_LIB; else export FDDM_HIP_LIB=$PWD/abl/$v.so; fi
  echo "== $v" >> gpurun_out/r06_t33_kl.txt
  timeout -k 10 120 python -u tools/kl_time.py >> gpurun_out/r06_t33_kl.txt 2>&1 || exit 1
done
echo done
