#!/bin/bash
# round-6 final tree: full GPU suite, smoke, bench line + kernel trace (measure.sh), C4 line
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06_t36_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_t36_smoke.log 2>&1 || exit 1
bash tools/measure.sh r06h || exit 1
timeout -k 10 400 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/r06h_c4.json 2> gpurun_out/r06h_c4.err || exit 1
echo done
