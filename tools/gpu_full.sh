#!/bin/bash
# One GPU call: GPU test files (stop at first crash/timeout), smoke(), default bench line, 2-rank launcher rehearsal.
mkdir -p gpurun_out
bash tools/gpu_run.sh tests/test_gpu_bench_parity.py tests/test_gpu_c5.py tests/test_gpu_step_configs.py tests/test_gpu_dist.py tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_sampler.py tests/test_gpu_e2e.py || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo bench failed; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
FDDM_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo gloo2 bench failed; tail -20 gpurun_out/bench_gloo2.err; exit 1; }
cat gpurun_out/bench_gloo2.json
