#!/bin/bash
# conditioning Linears: register-tile kernel only where it makes >= 128 blocks (FiLM), round-2 blocks elsewhere
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "small_linear or rows_mean" --timeout 120 --timeout-method thread > gpurun_out/r06_t28_k.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/cond_bench.py > gpurun_out/r06_t28_cond.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t28_parity.log 2>&1 || exit 1
bash tools/measure.sh r06g || exit 1
echo done
