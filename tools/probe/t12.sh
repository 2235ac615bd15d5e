set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5.py -v -k full_batch --timeout 500 --timeout-method thread > gpurun_out/t_c5b64.log 2>&1; r=$?
grep -E "PASS|FAIL|^E |passed|failed" gpurun_out/t_c5b64.log | head; exit $r
