#!/bin/bash
# bench.py under per-part encoder caps: "<conv1 cap> <conv2.. cap> <rest cap>" triples
for t in "$@"; do
  set -- $t
  FDDM_ENC_CUS_CONV=$1 FDDM_ENC_CUS_CONV2=$2 FDDM_ENC_CUS=$3 timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/cap2_$1_$2_$3.json 2> gpurun_out/cap2_$1_$2_$3.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/cap2_$1_$2_$3.json').read().strip().splitlines()[-1]);print('conv1 $1 conv2.. $2 rest $3:', d['value'], d['ms_per_step'])"
done
