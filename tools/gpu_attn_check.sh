#!/bin/bash
# One GPU call: attention kernel tests (default, and the streamed dQ kernel), attention micro-benchmark.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -k "attention" -p no:cacheprovider --tb=short --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
FDDM_ATTN_DQ2=1 FDDM_ATTN_DKV2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -k "attention" -p no:cacheprovider --tb=short --timeout 120 --timeout-method thread > gpurun_out/attn_tests_dq2.log 2>&1
rc=$?; tail -3 gpurun_out/attn_tests_dq2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; cat gpurun_out/attn_bench.log; exit $rc
