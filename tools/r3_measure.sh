set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || exit 1
cat gpurun_out/r03a_bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03a_trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03a_trace.log 2>&1 || exit 1
bash tools/pmc_conv1.sh gpurun_out/r03_pmc_conv1.json || exit 1
