#!/bin/bash
# Round 6 final tree after the KL reduction change: the train-step suites that run the fused KL, and smoke()
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
bash tools/gpu_run.sh tests/test_gpu_step_configs.py tests/test_gpu_step_graph.py tests/test_gpu_dist.py tests/test_gpu_models.py tests/test_gpu_e2e.py tests/test_gpu_c5.py tests/test_gpu_sampler.py > gpurun_out/r06_t56.txt 2>&1 || { cat gpurun_out/r06_t56.txt; exit 1; }
grep -E "rc=|passed|failed" gpurun_out/r06_t56.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_t56_smoke.log 2>&1 || { tail -20 gpurun_out/r06_t56_smoke.log; exit 1; }
tail -n 1 gpurun_out/r06_t56_smoke.log
