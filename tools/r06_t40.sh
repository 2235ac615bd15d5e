#!/bin/bash
# Round 6, session 2: conv-1 PMC traffic on the current kernel sources + a default bench line (box calibration).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06i_bench.json 2> gpurun_out/r06i_bench.err || exit 1
cat gpurun_out/r06i_bench.json
bash tools/pmc_conv1.sh gpurun_out/r06i_pmc_conv1.json || exit 1
cat gpurun_out/r06i_pmc_conv1.json
