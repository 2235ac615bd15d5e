#!/bin/bash
# HBM-bound kernels in isolation (LN, KL) and a same-box A/B of the RoPE-fused input gradient
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 120 python -u tools/ln_bench.py > gpurun_out/r06_t15_ln.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/kl_time.py > gpurun_out/r06_t15_kl.txt 2>&1 || exit 1
ROUNDS=3 bash tools/ab.sh - "FDDM_ROPE_FUSE=0" > gpurun_out/r06_t15_ab.txt 2>&1 || exit 1
echo done
