#!/bin/bash
# Round 6, session 2: keep-bit producer v2 (packed compares, bit transpose by DPP / permlane16_swap): parity, timing
# against the previous producer (abl/dmask_old.so), same-box step A/B; conv-1 PMC traffic + a default bench line.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "drop_bits or dropout" > gpurun_out/r06_t42_test.log 2>&1 || { tail -30 gpurun_out/r06_t42_test.log; exit 1; }
tail -2 gpurun_out/r06_t42_test.log
timeout -k 10 120 python -u tools/dmask_time.py new > gpurun_out/r06_t42_dm.txt 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/dmask_old.so timeout -k 10 120 python -u tools/dmask_time.py old >> gpurun_out/r06_t42_dm.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r06_t42_dm.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn7.py > gpurun_out/r06_t42_attn7.log 2>&1 || { tail -30 gpurun_out/r06_t42_attn7.log; exit 1; }
tail -2 gpurun_out/r06_t42_attn7.log
ROUNDS=3 bash tools/ab.sh - "FDDM_HIP_LIB=$PWD/abl/dmask_old.so" > gpurun_out/r06_t42_ab.txt 2>&1 || { cat gpurun_out/r06_t42_ab.txt; exit 1; }
cat gpurun_out/r06_t42_ab.txt
bash tools/pmc_conv1.sh gpurun_out/r06i_pmc_conv1.json || exit 1
cat gpurun_out/r06i_pmc_conv1.json
