#!/bin/bash
# fwd8 (two-chain forward) parity + timing
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_attn7.py > gpurun_out/r06_t3_attn.log 2>&1; rc=$?
timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,auto > gpurun_out/r06_t3_bench.log 2>&1
if [ $rc -eq 0 ]; then timeout -k 10 600 python -u tools/probe/rccl_diag.py > gpurun_out/r06_rccl_diag.log 2>&1; fi
echo "tests rc $rc"
exit $rc
