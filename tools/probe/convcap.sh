# C2 step at conv caps 128 (default) / 120 / 112 / 104 with the transformer cap 192, alternating (final round-5 tree:
# the encoder ends ~0.25 ms before the decoder, so fewer conv CUs might shorten the decoder's forward)
set -o pipefail
for r in 1 2 3; do
  for c in 128 120 112 104; do
    FDDM_ENC_CUS_CONV=$c timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline > /tmp/cs.json 2>/tmp/cs.err || { echo "failed $c"; tail -3 /tmp/cs.err; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/cs.json').read().strip().splitlines()[-1]);print('round $r conv $c:', d['value'], d['ms_per_step'])"
  done
done
