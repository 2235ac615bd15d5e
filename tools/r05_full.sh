#!/bin/bash
# One GPU call: the whole GPU test suite file by file, smoke(), bench C2 (with CPU baseline) and C4 lines.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r05}
bash tools/gpu_run.sh tests/test_gpu_attn7.py tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_bench_parity.py tests/test_gpu_step_configs.py tests/test_gpu_step_graph.py tests/test_gpu_dist.py tests/test_gpu_c5.py tests/test_gpu_sampler.py tests/test_gpu_e2e.py || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { echo bench failed; tail -20 gpurun_out/${TAG}_bench_default.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/${TAG}_bench_c4.json 2> gpurun_out/${TAG}_bench_c4.err || { echo c4 bench failed; tail -20 gpurun_out/${TAG}_bench_c4.err; exit 1; }
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
for f in (f"gpurun_out/{t}_bench_default.json", f"gpurun_out/{t}_bench_c4.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["host_ms_per_step"],
          {k: (v.get("kernel_us"), v.get("kernel_frac")) for k, v in d["decoder_attention"].items()})
PY
