#!/bin/bash
# round 6, first GPU call: the new parity tests (fwd7 slow path without a reference, RCCL world-1 forced DP, fused
# backward Lq cap) and the decoder attention bench on this box
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_attn7.py > gpurun_out/r06_t1_attn7.log 2>&1 || { echo attn7 tests failed; exit 1; }
timeout -k 10 120 python -u tools/attn7_bench.py 20 > gpurun_out/r06_t1_bench.log 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 650 --timeout-method thread tests/test_gpu_dist.py -k rccl > gpurun_out/r06_t1_rccl.log 2>&1 || { echo rccl failed; exit 1; }
echo done
