#!/bin/bash
# One GPU call: attention kernel tests (default and FDDM_ATTN_NW=16 forward), attention micro-benchmark.
mkdir -p gpurun_out
true
rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
true
rc=$?; tail -3 gpurun_out/attn_tests16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; cat gpurun_out/attn_bench.log; exit $rc
