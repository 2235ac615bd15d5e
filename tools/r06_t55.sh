#!/bin/bash
# Round 6: fused KL block reductions on DPP / permlane swaps (tree) vs __shfl_xor (ds_bpermute, abl/kl_shfl.so): KL
# parity, alternating timing (tools/kl_time.py), same-box step A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "kl or KL" > gpurun_out/r06_t55_k.log 2>&1 || { tail -30 gpurun_out/r06_t55_k.log; exit 1; }
echo "kl tests: $(tail -n 1 gpurun_out/r06_t55_k.log)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench_parity.py > gpurun_out/r06_t55_bp.log 2>&1 || { tail -30 gpurun_out/r06_t55_bp.log; exit 1; }
echo "bench parity: $(tail -n 1 gpurun_out/r06_t55_bp.log)"
out=gpurun_out/r06_t55.txt
: > $out
for r in 1 2 3; do
  echo "== round $r: dpp (tree)" >> $out
  timeout -k 10 120 python -u tools/kl_time.py 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  echo "== round $r: shfl (abl/kl_shfl.so)" >> $out
  FDDM_HIP_LIB=$PWD/abl/kl_shfl.so timeout -k 10 120 python -u tools/kl_time.py 2>&1 | grep -v amdgpu.ids >> $out || exit 1
done
cat $out
ROUNDS=3 bash tools/ab.sh - "FDDM_HIP_LIB=$PWD/abl/kl_shfl.so" > gpurun_out/r06_t55_ab.txt 2>&1 || { cat gpurun_out/r06_t55_ab.txt; exit 1; }
cat gpurun_out/r06_t55_ab.txt
