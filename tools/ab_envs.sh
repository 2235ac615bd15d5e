#!/bin/bash
# bench.py A/B over "VAR=value" settings (or "-" for none), alternating, on one box
mkdir -p gpurun_out
i=0
for kv in "$@"; do
  i=$((i+1))
  if [ "$kv" = "-" ]; then envs=""; else envs="$kv"; fi
  env $envs timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/abe_$i.json 2> gpurun_out/abe_$i.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abe_$i.json').read().strip().splitlines()[-1]);print('$kv', d['value'], d['ms_per_step'])"
done
