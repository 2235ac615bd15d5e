#!/bin/bash
# fwd8 v5: Q staged in the wave's private LDS (no barrier after its reads), epilogue stores from registers (permlane32 pairs,
# no LDS staging / barrier), private fallback staging: parity, timing (fwd7 / auto / fwd8), stamps
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn7.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_t20_attn7.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,fwd8 > gpurun_out/r06_t20_bench.log 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/a8st.so timeout -k 10 120 python -u tools/probe/a8_stamps.py > gpurun_out/r06_t20_stamps.log 2>&1 || exit 1
echo done
