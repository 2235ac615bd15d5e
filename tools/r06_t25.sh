#!/bin/bash
# C4 bench line on the round-6 tree; LN backward in the step's partials form
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 120 python -u tools/ln_bench.py > gpurun_out/r06_t25_ln.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/r06_t25_c4.json 2> gpurun_out/r06_t25_c4.err || exit 1
echo done
