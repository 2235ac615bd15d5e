# C2 step at a few encoder CU caps (FDDM_ENC_CUS / FDDM_ENC_CUS_CONV), alternating, after the fused attention backward
set -o pipefail
for r in 1 2; do
  for cfg in "192 128" "208 128" "192 144" "208 144" "176 128"; do
    set -- $cfg
    FDDM_ENC_CUS=$1 FDDM_ENC_CUS_CONV=$2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > /tmp/cs.json 2>/tmp/cs.err || { echo "failed $cfg"; tail -3 /tmp/cs.err; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/cs.json').read().strip().splitlines()[-1]);print('round $r enc $1 conv $2:', d['value'], d['ms_per_step'])"
  done
done
