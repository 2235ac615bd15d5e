#!/bin/bash
# Step time vs the encoder stream's persistent-GEMM CU cap (FDDM_ENC_CUS), one box.
for c in "$@"; do
  FDDM_ENC_CUS=$c timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 --warmup 4 > gpurun_out/sweep_$c.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sweep_$c.json'));print('$c', d['ms_per_step'], d['value'])"
done
