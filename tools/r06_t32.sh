#!/bin/bash
# fused KL: raw log2 per float4; 256- vs 512-thread rows
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q -k "kl" --timeout 120 --timeout-method thread > gpurun_out/r06_t32_k.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/kl_time.py > gpurun_out/r06_t32_kl.txt 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/kl512.so timeout -k 10 120 python -u tools/kl_time.py >> gpurun_out/r06_t32_kl.txt 2>&1 || exit 1
echo done
