#!/bin/bash
# GPU tests (kernels, models, step configs), then bench A/B: current library vs vlib/gelu_old.so, alternating
mkdir -p gpurun_out
bash tools/gpu_run.sh tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_step_configs.py tests/test_gpu_e2e.py || exit $?
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export FDDM_HIP_LIB=vlib/gelu_old.so; else unset FDDM_HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/ab_$lib$i.json 2> gpurun_out/ab_$lib$i.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$lib$i.json').read().strip().splitlines()[-1]);print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline_isolated']['avg_ms'])"
  done
done
