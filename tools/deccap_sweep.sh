#!/bin/bash
# bench.py under FDDM_DEC_CUS values (a probe that set the decoder launches' persistent-GEMM cap at the start of
# train_one_epoch; measured in round 2 and removed — DESIGN §4.2)
mkdir -p gpurun_out
for v in "$@"; do
  FDDM_DEC_CUS=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/dc_$v.json 2> gpurun_out/dc_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/dc_$v.json').read().strip().splitlines()[-1]);print('dec cap $v:', d['value'], d['ms_per_step'])"
done
