#!/bin/bash
# Round 6, session 2: WavLM attention on fwd7's bias build (attn7.hip REL): parity vs fwd5 and float64, timing of both
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wavlm_attention_fwd7 or relbias or relgate" > gpurun_out/r06_t44_test.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r06_t44_test.log | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/r06_t44_test.log
timeout -k 10 120 python -u tools/wavlm_attn_time.py > gpurun_out/r06_t44_time.txt 2>&1 || { cat gpurun_out/r06_t44_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_t44_time.txt
