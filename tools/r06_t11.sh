#!/bin/bash
# fwd8 with integer LDS addresses / 24-bit source offsets in the fill pieces: parity, timing, stamps; RCCL world-1 test
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn7.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_t11_attn7.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,auto > gpurun_out/r06_t11_bench.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v -k rccl --timeout 240 --timeout-method thread > gpurun_out/r06_t11_rccl.log 2>&1 || exit 1
echo done
