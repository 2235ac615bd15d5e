#!/bin/bash
# bench.py under FDDM_G128_NCU values (the CU count the grouped weight-gradient split choice assumes)
mkdir -p gpurun_out
for v in "$@"; do
  FDDM_G128_NCU=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/ncu_$v.json 2> gpurun_out/ncu_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ncu_$v.json').read().strip().splitlines()[-1]);print('ncu $v:', d['value'], d['ms_per_step'])"
done
