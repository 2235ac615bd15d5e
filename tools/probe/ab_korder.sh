# A/B: gemm256 conv K-tile order (vlib/korder.so, -DG256_KORDER) against the in-tree library; conv parity first
set -o pipefail
mkdir -p gpurun_out
FDDM_HIP_LIB=vlib/korder.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv" > gpurun_out/ko_tests.log 2>&1 || { tail -30 gpurun_out/ko_tests.log; exit 1; }
tail -1 gpurun_out/ko_tests.log
for r in 1 2; do
  timeout -k 10 120 python -u tools/conv_bench.py 10 > gpurun_out/ko_base$r.txt 2>&1 || exit 1
  FDDM_HIP_LIB=vlib/korder.so timeout -k 10 120 python -u tools/conv_bench.py 10 > gpurun_out/ko_var$r.txt 2>&1 || exit 1
done
for f in base1 var1 base2 var2; do echo "== $f"; grep -v amdgpu.ids gpurun_out/ko_$f.txt; done
