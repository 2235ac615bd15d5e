# fwd7 with both halves' K fragments read at the start of a tile (vlib/kpre.so, -DA7_KPRE) vs in-tree; parity of the
# variant first (attn7 tests), then attn7_bench alternating
set -o pipefail
FDDM_HIP_LIB=vlib/kpre.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn7.py > /tmp/kp.log 2>&1 || { tail -20 /tmp/kp.log; exit 1; }
tail -1 /tmp/kp.log
for r in 1 2; do
  for lib in fddm-asr_amd/fddm_hip/libfddm_hip.so vlib/kpre.so; do
    echo "== $r $lib"; FDDM_HIP_LIB=$lib timeout -k 10 120 python -u tools/attn7_bench.py 50 2>&1 | grep "C2\|C4" | sed 's/v6: .* | auto/auto/; s/bwd .*//' || exit 1
  done
done
