#!/bin/bash
for v in default nopersist default nopersist; do
  if [ $v = default ]; then unset FDDM_HIP_LIB; else export FDDM_HIP_LIB=$PWD/variants/$v.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 --warmup 4 > gpurun_out/var_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/var_$v.json'));print('$v', d['ms_per_step'], d['value'])"
done
