#!/bin/bash
# Round-end measurement call: every GPU test file, smoke(), the default bench line, the 2-rank gloo rehearsal,
# a rocprofv3 kernel-trace/stats pass over the bench, then the PMC passes (traffic + SQ counters).
# Usage: bash tools/gpu_measure.sh <tag>
tag=${1:-r02e}
export TMPDIR=/tmp
bash tools/gpu_full.sh || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1 || { echo "kernel-trace pass failed"; tail -5 gpurun_out/prof_$tag.log; exit 1; }
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
python3 tools/prof_summary.py "$f" 45 > gpurun_out/prof_${tag}_top.txt && head -30 gpurun_out/prof_${tag}_top.txt
bash tools/pmc_passes.sh $tag
