set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn7.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_attn7.log 2>&1
rc=$?
tail -30 gpurun_out/t_attn7.log
exit $rc
