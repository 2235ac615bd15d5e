#!/bin/bash
# Round 6, session 2: keep-bit producer v3 (single ds_read_b64 gathers by hand): parity + timing against abl/dmask_old.so
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "drop_bits or dropout" > gpurun_out/r06_t43_test.log 2>&1 || { tail -30 gpurun_out/r06_t43_test.log; exit 1; }
tail -1 gpurun_out/r06_t43_test.log
timeout -k 10 120 python -u tools/dmask_time.py new > gpurun_out/r06_t43_dm.txt 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/dmask_old.so timeout -k 10 120 python -u tools/dmask_time.py old >> gpurun_out/r06_t43_dm.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r06_t43_dm.txt
