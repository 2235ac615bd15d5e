#!/bin/bash
# One GPU call: kernel + model GPU tests (stop on crash/timeout), then the micro-benchmarks named as arguments.
mkdir -p gpurun_out
bash tools/gpu_run.sh tests/test_gpu_kernels.py tests/test_gpu_models.py || exit $?
for t in "$@"; do
  timeout -k 10 180 python -u $t > gpurun_out/$(basename $t .py).log 2>&1; rc=$?; cat gpurun_out/$(basename $t .py).log; [ $rc -eq 0 ] || exit $rc
done
