#!/bin/bash
# Round 6, session 2: new keep-bit producer (packed compares + bit transpose): parity, timing vs the previous producer;
# conv-1 PMC traffic on the current kernel sources + a default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "drop_bits or dropout" > gpurun_out/r06_t41_test.log 2>&1 || { tail -30 gpurun_out/r06_t41_test.log; exit 1; }
tail -3 gpurun_out/r06_t41_test.log
timeout -k 10 120 python -u tools/dmask_time.py new > gpurun_out/r06_t41_dm.txt 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/dmask_old.so timeout -k 10 120 python -u tools/dmask_time.py old >> gpurun_out/r06_t41_dm.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/dmask_time.py new >> gpurun_out/r06_t41_dm.txt 2>&1 || exit 1
cat gpurun_out/r06_t41_dm.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn7.py > gpurun_out/r06_t41_attn7.log 2>&1 || { tail -30 gpurun_out/r06_t41_attn7.log; exit 1; }
tail -2 gpurun_out/r06_t41_attn7.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06i_bench.json 2> gpurun_out/r06i_bench.err || exit 1
cat gpurun_out/r06i_bench.json
bash tools/pmc_conv1.sh gpurun_out/r06i_pmc_conv1.json || exit 1
cat gpurun_out/r06i_pmc_conv1.json
