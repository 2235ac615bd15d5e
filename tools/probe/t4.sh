set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn7.py -v -k rescale --timeout 120 --timeout-method thread > gpurun_out/t_attn7r.log 2>&1
grep -E "PASS|FAIL|max err" gpurun_out/t_attn7r.log | head -40
