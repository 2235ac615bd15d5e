#!/bin/bash
# Round 6, session 2 final tree (r06j: before the gemm256 epilogue change; r06m: after): every GPU test file, smoke(), the default C2 bench line (with the CPU baseline), the
# C4 line, and a rocprofv3 kernel trace of the C2 bench (tools/measure.sh layout) -> gpurun_out/r06m_*
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
bash tools/gpu_run.sh tests/test_gpu_kernels.py tests/test_gpu_attn7.py tests/test_gpu_models.py tests/test_gpu_e2e.py tests/test_gpu_sampler.py tests/test_gpu_c5.py tests/test_gpu_step_configs.py tests/test_gpu_step_graph.py tests/test_gpu_dist.py tests/test_gpu_bench_parity.py > gpurun_out/r06m_tests.txt 2>&1 || { cat gpurun_out/r06m_tests.txt; exit 1; }
grep -E "rc=|passed|failed" gpurun_out/r06m_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06m_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r06m_smoke.log; exit 1; }
tail -n 2 gpurun_out/r06m_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r06m_bench_default.json 2> gpurun_out/r06m_bench_default.err || { tail -20 gpurun_out/r06m_bench_default.err; exit 1; }
cat gpurun_out/r06m_bench_default.json
timeout -k 10 600 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/r06m_bench_c4.json 2> gpurun_out/r06m_bench_c4.err || { tail -20 gpurun_out/r06m_bench_c4.err; exit 1; }
cat gpurun_out/r06m_bench_c4.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06m_trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06m_trace.log 2>&1 || exit 1
tail -c 300 gpurun_out/r06m_trace.log
