set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn7.py -q --timeout 120 --timeout-method thread > gpurun_out/t_attn7d.log 2>&1; r=$?
tail -3 gpurun_out/t_attn7d.log; grep -E "^E " gpurun_out/t_attn7d.log | head
[ $r -eq 0 ] || exit $r
for lib in vlib/a7old.so fddm-asr_amd/fddm_hip/libfddm_hip.so vlib/a7old.so fddm-asr_amd/fddm_hip/libfddm_hip.so; do
  echo "== $lib"; FDDM_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python -u tools/attn7_bench.py 50 2>&1 | grep -v amdgpu.ids | sed 's/v6:.*| auto/auto/' || exit 1
done
