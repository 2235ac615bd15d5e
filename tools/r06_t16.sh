#!/bin/bash
# LN backward with every row of a wave loaded up front: kernel tests + micro-benchmark
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "layernorm or ln_" --timeout 120 --timeout-method thread > gpurun_out/r06_t16_ln_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/ln_bench.py > gpurun_out/r06_t16_ln.txt 2>&1 || exit 1
echo done
