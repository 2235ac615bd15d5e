set -o pipefail
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -k "small_linear" --timeout 120 --timeout-method thread 2>&1 | tail -3
for v in smallold - smallold -; do
  if [ "$v" = "-" ]; then lib=""; else lib="FDDM_HIP_LIB=$GRAFT_REPO_ROOT/vlib/$v.so"; fi
  echo "== $v"; env $lib timeout -k 10 100 python -u tools/probe/small_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
