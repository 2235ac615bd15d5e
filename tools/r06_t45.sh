#!/bin/bash
# Round 6, session 2: WavLM attention on fwd7's bias build (packed bias FMAs / row sums) + keep-bit producer v3:
# kernel, model and bench-path parity, WavLM attention timing, then a same-box step A/B against fwd5
# (FDDM_ATTN_KERNELS=relfwd5)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wavlm_attention_fwd7 or relbias or relgate" > gpurun_out/r06_t45_k.log 2>&1 || { tail -30 gpurun_out/r06_t45_k.log; exit 1; }
echo "kernels: $(tail -n 1 gpurun_out/r06_t45_k.log)"
timeout -k 10 120 python -u tools/wavlm_attn_time.py > gpurun_out/r06_t45_time.txt 2>&1 || { cat gpurun_out/r06_t45_time.txt; exit 1; }
echo "four shifted copies (abl/rel4copies.so):" >> gpurun_out/r06_t45_time.txt
FDDM_HIP_LIB=$PWD/abl/rel4copies.so timeout -k 10 120 python -u tools/wavlm_attn_time.py >> gpurun_out/r06_t45_time.txt 2>&1 || { cat gpurun_out/r06_t45_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_t45_time.txt
for t in test_gpu_attn7 test_gpu_models test_gpu_e2e test_gpu_bench_parity; do
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/$t.py > gpurun_out/r06_t45_$t.log 2>&1 || { tail -30 gpurun_out/r06_t45_$t.log; exit 1; }
  echo "$t: $(tail -n 1 gpurun_out/r06_t45_$t.log)"
done
ROUNDS=3 bash tools/ab.sh - "FDDM_ATTN_KERNELS=relfwd5" > gpurun_out/r06_t45_ab.txt 2>&1 || { cat gpurun_out/r06_t45_ab.txt; exit 1; }
cat gpurun_out/r06_t45_ab.txt
