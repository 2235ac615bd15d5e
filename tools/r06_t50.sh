#!/bin/bash
# Round 6, session 2: gemm256 epilogue lane exchanges without lane-parity selects (chunk16 as one v_permlane16_swap of
# the two packed blocks): GEMM parity (kernel tests, WavLM fixtures, bench path), GEMM / conv timing against the previous
# gemm256 (abl/g256old.so), a same-box step A/B, and the conv-1 PMC traffic of the new kernel sources
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/r06_t50_k.log 2>&1 || { tail -30 gpurun_out/r06_t50_k.log; exit 1; }
echo "kernels: $(tail -n 1 gpurun_out/r06_t50_k.log)"
for t in test_gpu_models test_gpu_e2e test_gpu_bench_parity; do
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/$t.py > gpurun_out/r06_t50_$t.log 2>&1 || { tail -30 gpurun_out/r06_t50_$t.log; exit 1; }
  echo "$t: $(tail -n 1 gpurun_out/r06_t50_$t.log)"
done
out=gpurun_out/r06_t50.txt
: > $out
for r in 1 2; do
  echo "== round $r: tree" >> $out
  timeout -k 10 180 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  timeout -k 10 180 python -u tools/conv_bench.py 10 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  echo "== round $r: previous gemm256 (abl/g256old.so)" >> $out
  FDDM_HIP_LIB=$PWD/abl/g256old.so timeout -k 10 180 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  FDDM_HIP_LIB=$PWD/abl/g256old.so timeout -k 10 180 python -u tools/conv_bench.py 10 2>&1 | grep -v amdgpu.ids >> $out || exit 1
done
cat $out
ROUNDS=3 bash tools/ab.sh - "FDDM_HIP_LIB=$PWD/abl/g256old.so" > gpurun_out/r06_t50_ab.txt 2>&1 || { cat gpurun_out/r06_t50_ab.txt; exit 1; }
cat gpurun_out/r06_t50_ab.txt
bash tools/pmc_conv1.sh gpurun_out/r06k_pmc_conv1.json || exit 1
cat gpurun_out/r06k_pmc_conv1.json
