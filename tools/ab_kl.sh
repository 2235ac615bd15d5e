#!/bin/bash
# KL kernel tests, then tools/kl_bench.py on the current library and on vlib/kl_old.so (same box)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -q -m gpu -p no:cacheprovider --tb=short --timeout 120 --timeout-method thread > gpurun_out/kl_tests.log 2>&1; rc=$?; tail -3 gpurun_out/kl_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/kl_bench.py && FDDM_HIP_LIB=vlib/kl_old.so timeout -k 10 120 python -u tools/kl_bench.py
