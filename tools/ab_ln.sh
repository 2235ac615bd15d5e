bash tools/gpu_quick.sh tools/ln_bench.py && FDDM_HIP_LIB=vlib/ln_old.so timeout -k 10 120 python -u tools/ln_bench.py
