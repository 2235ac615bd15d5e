#!/bin/bash
# A/B of bench.py on one box: each argument is an env assignment list ("" = defaults), run in order
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$i.json').read().strip().splitlines()[-1]);print('[$envs]:', d['value'], d['ms_per_step'])"
done
