#!/bin/bash
# fwd8 v6: row sums by row-selector MFMAs into one accumulator shared by the chains: parity, timing against fwd7 and
# the f32-add build (abl/rsadd.so), stamps
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn7.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_t21_attn7.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,fwd8 > gpurun_out/r06_t21_bench.log 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/a8st.so timeout -k 10 120 python -u tools/probe/a8_stamps.py > gpurun_out/r06_t21_stamps.log 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/rsadd.so timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd8 > gpurun_out/r06_t21_bench_rsadd.log 2>&1 || exit 1
echo done
