# conv K-tile orders: tap-major (in-tree) vs taps 0,2,1 per channel block (vlib/korder.so) vs taps 0/2 interleaved
# first, then tap 1 (vlib/korder2.so, bit-op index map); conv parity under korder2, then alternating conv_bench runs
set -o pipefail
FDDM_HIP_LIB=vlib/korder2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv" > /tmp/k.log 2>&1 || { tail -20 /tmp/k.log; exit 1; }
tail -1 /tmp/k.log
for r in 1 2; do
  for lib in fddm-asr_amd/fddm_hip/libfddm_hip.so vlib/korder.so vlib/korder2.so; do
    echo "== $r $lib"; FDDM_HIP_LIB=$lib timeout -k 10 120 python -u tools/conv_bench.py 10 2>&1 | grep -v amdgpu.ids | grep "conv1 \|total" || exit 1
  done
done
