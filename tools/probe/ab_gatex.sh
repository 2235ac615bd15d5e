# WavLM gate in the attention kernel from x (default "x") vs extra Q|K|V columns ("cols"): parity, then alternating
# C2 bench runs
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "relgate or wavlm or conv" > /tmp/g1.log 2>&1 || { tail -30 /tmp/g1.log; exit 1; }
tail -1 /tmp/g1.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_bench_parity.py > /tmp/g2.log 2>&1 || { tail -30 /tmp/g2.log; exit 1; }
tail -1 /tmp/g2.log
for r in 1 2 3; do
  for v in cols x; do
    FDDM_WAVLM_GATE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > /tmp/ab.json 2>/tmp/ab.err || { echo "failed $v"; tail -3 /tmp/ab.err; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]);print('round $r gate=$v:', d['value'], d['ms_per_step'])"
  done
done
