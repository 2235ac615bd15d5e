set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread > gpurun_out/t_dist.log 2>&1; r=$?
grep -E "PASS|FAIL|^E " gpurun_out/t_dist.log | head -40
exit $r
