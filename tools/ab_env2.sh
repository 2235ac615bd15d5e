#!/bin/bash
# GPU tests, then bench A/B of an env toggle, alternating on one box. Usage: bash tools/ab_env2.sh VAR A B
var=$1; a=$2; b=$3
mkdir -p gpurun_out
bash tools/gpu_run.sh tests/test_gpu_step_configs.py tests/test_gpu_models.py tests/test_gpu_e2e.py tests/test_gpu_dist.py tests/test_gpu_sampler.py || exit $?
for i in 1 2; do
  for v in $a $b; do
    env $var=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/ab2_$v$i.json 2> gpurun_out/ab2_$v$i.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab2_$v$i.json').read().strip().splitlines()[-1]);print('$var=$v', d['value'], d['ms_per_step'])"
  done
done
