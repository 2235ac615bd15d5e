#!/bin/bash
# Round 6, session 2: fwd7 with packed f32 adds / FMAs (bias, row sums: the tree) vs scalar (abl/unpacked.so), WavLM
# shape and the decoder shapes (fwd7 family), two alternating rounds on one box
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
out=gpurun_out/r06_t48.txt
: > $out
for r in 1 2; do
  echo "== round $r: packed (tree)" >> $out
  timeout -k 10 120 python -u tools/wavlm_attn_time.py 2>&1 | grep auto >> $out || exit 1
  timeout -k 10 180 python -u tools/attn7_bench.py 20 fwd7 2>&1 | grep -v amdgpu.ids >> $out || exit 1
  echo "== round $r: scalar (abl/unpacked.so)" >> $out
  FDDM_HIP_LIB=$PWD/abl/unpacked.so timeout -k 10 120 python -u tools/wavlm_attn_time.py 2>&1 | grep auto >> $out || exit 1
  FDDM_HIP_LIB=$PWD/abl/unpacked.so timeout -k 10 180 python -u tools/attn7_bench.py 20 fwd7 2>&1 | grep -v amdgpu.ids >> $out || exit 1
done
cat $out
