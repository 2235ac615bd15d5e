#!/bin/bash
# Round 6 second session as a whole: the final tree against the session's starting library (abl/r06h.so: attn7.hip,
# attention.hip and gemm256.hip of commit ddbeee3), same box, alternating; C2 (4 rounds) and C4 (2 rounds)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
ROUNDS=4 bash tools/ab.sh - "FDDM_HIP_LIB=$PWD/abl/r06h.so" > gpurun_out/r06_t52_c2.txt 2>&1 || { cat gpurun_out/r06_t52_c2.txt; exit 1; }
cat gpurun_out/r06_t52_c2.txt
ROUNDS=2 BENCH_ARGS="--config c4" bash tools/ab.sh - "FDDM_HIP_LIB=$PWD/abl/r06h.so" > gpurun_out/r06_t52_c4.txt 2>&1 || { cat gpurun_out/r06_t52_c4.txt; exit 1; }
cat gpurun_out/r06_t52_c4.txt
