set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "producer" -v --timeout 120 --timeout-method thread > gpurun_out/t_prod.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn7.py -v --timeout 120 --timeout-method thread > gpurun_out/t_attn7c.log 2>&1
grep -E "PASS|FAIL|Error|error" gpurun_out/t_prod.log | head -20; grep -E "PASS|FAIL" gpurun_out/t_attn7c.log | head -40
