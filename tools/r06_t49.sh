#!/bin/bash
# Round 6, session 2: the MFMA GEMM kernels (gemm256 / gemm128 / posconv) without SLP-vectorised packed f32 epilogue
# arithmetic (abl/noslp.so) vs the tree: GEMM micro-benchmark, conv layers, then a same-box step A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
out=gpurun_out/r06_t49.txt
: > $out
for r in 1 2; do
  echo "== round $r: tree" >> $out
  timeout -k 10 180 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  timeout -k 10 180 python -u tools/conv_bench.py 10 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  echo "== round $r: no SLP (abl/noslp.so)" >> $out
  FDDM_HIP_LIB=$PWD/abl/noslp.so timeout -k 10 180 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  FDDM_HIP_LIB=$PWD/abl/noslp.so timeout -k 10 180 python -u tools/conv_bench.py 10 2>&1 | grep -v amdgpu.ids >> $out || exit 1
done
cat $out
ROUNDS=3 bash tools/ab.sh - "FDDM_HIP_LIB=$PWD/abl/noslp.so" > gpurun_out/r06_t49_ab.txt 2>&1 || { cat gpurun_out/r06_t49_ab.txt; exit 1; }
cat gpurun_out/r06_t49_ab.txt
