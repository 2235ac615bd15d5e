set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn7.py -v --timeout 120 --timeout-method thread > gpurun_out/t_attn7c.log 2>&1; r=$?
grep -E "PASS|FAIL|^E " gpurun_out/t_attn7c.log | head -40
[ $r -eq 0 ] || exit $r
timeout -k 10 200 python -u tools/attn7_bench.py 50 2>&1 | grep -v amdgpu.ids
