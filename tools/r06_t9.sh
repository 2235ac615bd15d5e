#!/bin/bash
# fwd8 v3: prologue with Q by LDS-DMA before the key mask, two prologue tiles, fills spread over the spans
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_attn7.py > gpurun_out/r06_t9_attn.log 2>&1 || { echo attn tests failed; exit 1; }
timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,auto > gpurun_out/r06_t9_bench.log 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/a8st.so timeout -k 10 120 python -u tools/probe/a8_stamps.py > gpurun_out/r06_t9_stamps.log 2>&1 || exit 1
echo done
