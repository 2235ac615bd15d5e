#!/bin/bash
# Round 6: bwdf7's 8-lane delta sum on DPP (tree) vs __shfl_xor (abl/bwd_shfl.so): attention parity, alternating
# backward timing (tools/attn7_bench.py), same-box step A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn7.py > gpurun_out/r06_t57_k.log 2>&1 || { tail -30 gpurun_out/r06_t57_k.log; exit 1; }
echo "attn7: $(tail -n 1 gpurun_out/r06_t57_k.log)"
out=gpurun_out/r06_t57.txt
: > $out
for r in 1 2; do
  echo "== round $r: dpp (tree)" >> $out
  timeout -k 10 180 python -u tools/attn7_bench.py 20 auto 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  echo "== round $r: shfl (abl/bwd_shfl.so)" >> $out
  FDDM_HIP_LIB=$PWD/abl/bwd_shfl.so timeout -k 10 180 python -u tools/attn7_bench.py 20 auto 2>&1 | grep -v amdgpu.ids >> $out || exit 1
done
cat $out
ROUNDS=3 bash tools/ab.sh - "FDDM_HIP_LIB=$PWD/abl/bwd_shfl.so" > gpurun_out/r06_t57_ab.txt 2>&1 || { cat gpurun_out/r06_t57_ab.txt; exit 1; }
cat gpurun_out/r06_t57_ab.txt
