#!/bin/bash
# bench.py under encoder persistent-GEMM caps: "<conv cap> <rest cap>" pairs (0 = the default for that part)
for pair in "$@"; do
  set -- $pair
  FDDM_ENC_CUS_CONV=$1 FDDM_ENC_CUS=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/cap_$1_$2.json 2> gpurun_out/cap_$1_$2.err || exit 1
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/cap_$1_$2.json').read().strip().splitlines()[-1]);print('conv cap $1 rest cap $2:', d['value'], d['ms_per_step'])"
done
