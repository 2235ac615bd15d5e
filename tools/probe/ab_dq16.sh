# fused attention backward: dQ as two 16x16x32 blocks per wave on every tile (this library) against one 32x32x16
# block on the waves of the tile's parity (vlib/dq32.so); parity first, then attn7_bench alternating
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn7.py > gpurun_out/dq16_tests.log 2>&1 || { tail -40 gpurun_out/dq16_tests.log; exit 1; }
tail -1 gpurun_out/dq16_tests.log
for r in 1 2; do
  for lib in fddm-asr_amd/fddm_hip/libfddm_hip.so vlib/dq32.so; do
    echo "== $r $lib"; FDDM_HIP_LIB=$lib timeout -k 10 120 python -u tools/attn7_bench.py 50 2>&1 | grep "C2" | sed 's/v6: .* | auto/auto/' || exit 1
  done
done
