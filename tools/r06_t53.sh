#!/bin/bash
# Round 6: WavLM attention bias reads as single ds_read_b64 (tree) vs hipcc's ds_read2_b64 pairs (abl/rel_read2.so):
# parity, then alternating timing on one box, then a same-box step A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wavlm_attention_fwd7 or relbias or relgate" > gpurun_out/r06_t53_k.log 2>&1 || { tail -30 gpurun_out/r06_t53_k.log; exit 1; }
echo "kernels: $(tail -n 1 gpurun_out/r06_t53_k.log)"
out=gpurun_out/r06_t53.txt
: > $out
for r in 1 2 3; do
  echo "== round $r: b64 (tree)" >> $out
  timeout -k 10 120 python -u tools/wavlm_attn_time.py 2>&1 | grep auto >> $out || exit 1
  echo "== round $r: read2 (abl/rel_read2.so)" >> $out
  FDDM_HIP_LIB=$PWD/abl/rel_read2.so timeout -k 10 120 python -u tools/wavlm_attn_time.py 2>&1 | grep auto >> $out || exit 1
done
cat $out
ROUNDS=3 bash tools/ab.sh - "FDDM_HIP_LIB=$PWD/abl/rel_read2.so" > gpurun_out/r06_t53_ab.txt 2>&1 || { cat gpurun_out/r06_t53_ab.txt; exit 1; }
cat gpurun_out/r06_t53_ab.txt
