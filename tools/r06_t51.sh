#!/bin/bash
# Round 6 final tree: the C5 jumpy-sampler line (with its CPU baseline) and a rocprofv3 kernel trace of the C4 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --config c5 > gpurun_out/r06l_bench_c5.json 2> gpurun_out/r06l_bench_c5.err || { tail -20 gpurun_out/r06l_bench_c5.err; exit 1; }
cat gpurun_out/r06l_bench_c5.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06l_c4t -o run -- python3 bench.py --config c4 --steps 8 --warmup 4 --no-cpu-baseline > gpurun_out/r06l_c4t.log 2>&1 || exit 1
tail -c 300 gpurun_out/r06l_c4t.log
