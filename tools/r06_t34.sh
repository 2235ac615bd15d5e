#!/bin/bash
# fused KL at 4 waves per SIMD: KL tests, timing, bench-path parity
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q -k "kl" --timeout 120 --timeout-method thread > gpurun_out/r06_t34_k.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/kl_time.py > gpurun_out/r06_t34_kl.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t34_parity.log 2>&1 || exit 1
echo done
