mkdir -p gpurun_out
FDDM_ATTN_REL3=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -k "relbias or relgate" -p no:cacheprovider --tb=short --timeout 120 --timeout-method thread > gpurun_out/rel3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/rel3_tests.log
timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
