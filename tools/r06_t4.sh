#!/bin/bash
# fwd8 v2 (row-sum MFMA, keep-bit layout v5 with v_perm masks): parity, then timing vs fwd7, and the 1-WG/CU variant
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_attn7.py > gpurun_out/r06_t4_attn.log 2>&1 || { echo attn tests failed; exit 1; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "drop_bits or attention" > gpurun_out/r06_t4_kern.log 2>&1 || { echo kernel tests failed; exit 1; }
timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,auto > gpurun_out/r06_t4_bench.log 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/wg1.so timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,auto > gpurun_out/r06_t4_bench_wg1.log 2>&1 || exit 1

FDDM_HIP_LIB=$PWD/abl/a8st.so timeout -k 10 120 python -u tools/probe/a8_stamps.py > gpurun_out/r06_t4_stamps.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/fill_sources.py 2 > gpurun_out/r06_t4_fills.log 2>&1 || exit 1
echo done2
