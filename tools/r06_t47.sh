#!/bin/bash
# Round 6, session 2: keep-bit producer on a stream of its own (joined before block 0): decoder / bench-path parity,
# graph-replay test, then a same-box step A/B against the producer on the decoder's stream (FDDM_BITS_STREAM=0)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
for t in test_gpu_step_graph test_gpu_bench_parity; do
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/$t.py > gpurun_out/r06_t47_$t.log 2>&1 || { tail -30 gpurun_out/r06_t47_$t.log; exit 1; }
  echo "$t: $(tail -n 1 gpurun_out/r06_t47_$t.log)"
done
ROUNDS=3 bash tools/ab.sh - "FDDM_BITS_STREAM=0" > gpurun_out/r06_t47_ab.txt 2>&1 || { cat gpurun_out/r06_t47_ab.txt; exit 1; }
cat gpurun_out/r06_t47_ab.txt
