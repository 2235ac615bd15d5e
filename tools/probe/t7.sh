set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t_g128.log 2>&1; r=$?
grep -E "PASS|FAIL|^E " gpurun_out/t_g128.log | head -40
[ $r -eq 0 ] || exit $r
for lib in vlib/g128old.so fddm-asr_amd/fddm_hip/libfddm_hip.so; do
  echo "== $lib"
  FDDM_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python -u tools/dx_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
