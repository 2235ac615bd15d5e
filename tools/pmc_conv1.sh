#!/bin/bash
# Two PMC passes (FETCH_SIZE, WRITE_SIZE) over a short bench run, then per-launch HBM traffic of the conv-1
# implicit GEMM (tools/pmc_traffic.py). Usage: bash tools/pmc_conv1.sh <out.json>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE/run_counter_collection.csv gpurun_out/pmc_WRITE_SIZE/run_counter_collection.csv "gemm256_kernel<3" "$1" 32
