cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4t -o run -- python3 bench.py --config c4 --steps 8 --warmup 4 --no-cpu-baseline > gpurun_out/c4t.log 2>&1 || exit 1
tail -c 300 gpurun_out/c4t.log
