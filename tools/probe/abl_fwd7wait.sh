# timing-only ablation of fwd7's per-tile ring sync (results wrong by design, never used for parity): the in-tree
# forward vs no vmcnt(0) wait (vlib/abl_NOWAIT.so) vs no wait and no barrier (vlib/abl_NOBAR.so), fwd only
set -o pipefail
for r in 1 2; do
  for lib in fddm-asr_amd/fddm_hip/libfddm_hip.so vlib/abl_NOWAIT.so vlib/abl_NOBAR.so; do
    echo "== $r $lib"; FDDM_HIP_LIB=$lib timeout -k 10 120 python -u tools/attn7_bench.py 50 2>&1 | grep "C2\|C4" | sed 's/v6: .* | auto/auto/; s/bwd .*//' || exit 1
  done
done
