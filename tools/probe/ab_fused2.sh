# fused attention backward with key passes: parity, then tools/attn7_bench.py on this library, the previous one
# (vlib/base.so) and a variant taking the fused launch up to Lq 1024 (vlib/fq1024.so: C4's shapes too)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn7.py tests/test_gpu_kernels.py -k "attn or attention" > gpurun_out/fu_tests.log 2>&1 || { tail -40 gpurun_out/fu_tests.log; exit 1; }
tail -2 gpurun_out/fu_tests.log
timeout -k 10 120 python -u tools/attn7_bench.py 50 > gpurun_out/fu_new.txt 2>&1 && FDDM_HIP_LIB=vlib/base.so timeout -k 10 120 python -u tools/attn7_bench.py 50 > gpurun_out/fu_base.txt 2>&1 && FDDM_HIP_LIB=vlib/fq1024.so timeout -k 10 120 python -u tools/attn7_bench.py 50 > gpurun_out/fu_fq.txt 2>&1 && timeout -k 10 120 python -u tools/attn7_bench.py 50 > gpurun_out/fu_new2.txt 2>&1
for f in new base fq new2; do echo "== $f"; grep -v amdgpu.ids gpurun_out/fu_$f.txt | sed 's/v6: .* | auto/auto/'; done
