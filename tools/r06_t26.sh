#!/bin/bash
# rows_mean on 8x the blocks, no sqrt / loss-add launches per step: kernel + optimizer tests, bench-path parity, bench
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "rows_mean or clip or adamw" --timeout 120 --timeout-method thread > gpurun_out/r06_t26_k.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t26_parity.log 2>&1 || exit 1
bash tools/measure.sh r06e || exit 1
echo done
