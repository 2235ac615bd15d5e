set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn7.py tests/test_gpu_kernels.py -k "attn or attention" -x -v --timeout 120 --timeout-method thread > gpurun_out/t_attn7b.log 2>&1
rc=$?
tail -45 gpurun_out/t_attn7b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn7_bench.py > gpurun_out/attn7_bench.txt 2>&1; cat gpurun_out/attn7_bench.txt
