#!/bin/bash
# rope-fused self-attention input gradient: kernel test, decoder bench-path parity, C2 bench line
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "rope" --timeout 120 --timeout-method thread > gpurun_out/r06_t14_rope.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_t14_parity.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06_t14_bench.json 2> gpurun_out/r06_t14_bench.err || exit 1
timeout -k 10 200 python -u tools/timeline.py > gpurun_out/r06_t14_timeline.txt 2>&1 || exit 1
echo done
