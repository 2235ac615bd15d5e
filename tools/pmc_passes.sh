#!/bin/bash
# Counter passes over a short bench run (one rocprofv3 process per pass; a pass never mixes --pmc with tracing):
#   trace: --kernel-trace --stats      fetch: FETCH_SIZE      write: WRITE_SIZE
#   sq:    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE
# then tools/pmc_table.py joins them per (kernel, grid). Usage: bash tools/pmc_passes.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
args=${@:-"--steps 2 --warmup 1 --no-cpu-baseline"}
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/pmc_$tag
mkdir -p $out
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args > $out/trace.log 2>&1 || { echo "trace pass failed"; tail -5 $out/trace.log; exit 1; }
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/p$i -o run -- python3 bench.py $args > $out/p$i.log 2>&1 || { echo "pmc pass $i ($c) failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $out > $out/table.md && head -60 $out/table.md
