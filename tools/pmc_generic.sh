#!/bin/bash
# rocprofv3 counter passes over one command, one pass per counter group (groups separated by ':'), then a
# per-kernel table of every counter (tools/pmc_kernels.py). Usage:
#   bash tools/pmc_generic.sh <tag> "<c1 c2 ...>:<c3 ...>" <python script and args...>
set -o pipefail
tag=$1; groups=$2; shift 2
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/pmcg_$tag
mkdir -p $out
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 "$@" > $out/trace.log 2>&1 || { echo "trace pass failed"; tail -5 $out/trace.log; exit 1; }
IFS=':' read -ra G <<< "$groups"
i=0
for c in "${G[@]}"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $out/p$i -o run -- python3 "$@" > $out/p$i.log 2>&1 || { echo "pmc pass $i ($c) failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 tools/pmc_kernels.py $out > $out/table.md && cat $out/table.md
