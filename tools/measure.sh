#!/bin/bash
# Round measurement: default bench line + rocprofv3 kernel-trace/stats of the same command (+ conv-1 PMC traffic
# when PMC=1). Usage: bash tools/measure.sh TAG   -> gpurun_out/TAG_bench.json, gpurun_out/TAG_trace/
set -o pipefail
TAG=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_trace.log 2>&1 || exit 1
tail -c 300 gpurun_out/${TAG}_trace.log
if [ "${PMC:-0}" = 1 ]; then bash tools/pmc_conv1.sh gpurun_out/${TAG}_pmc_conv1.json || exit 1; fi
