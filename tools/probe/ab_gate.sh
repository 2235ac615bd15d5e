# WavLM gate: extra Q|K|V output columns (default) vs the separate gate kernel (FDDM_WAVLM_GATE_SEPARATE=1);
# parity of the bf16 encoder under the variant, then alternating C2 bench runs
set -o pipefail
FDDM_WAVLM_GATE_SEPARATE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py > /tmp/g.log 2>&1 || { tail -20 /tmp/g.log; exit 1; }
tail -1 /tmp/g.log
for r in 1 2 3; do
  for v in 0 1; do
    FDDM_WAVLM_GATE_SEPARATE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > /tmp/ab.json 2>/tmp/ab.err || { echo "failed $v"; tail -3 /tmp/ab.err; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]);print('round $r separate=$v:', d['value'], d['ms_per_step'])"
  done
done
