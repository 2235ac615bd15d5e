# Same-box A/B of the round-4 tree (git worktree r04tree at e9e7adc, its own library) against this tree: alternating
# default bench runs (C2), then C4.
set -o pipefail
for cfg in "" "--config c4"; do
for r in 1 2; do
  for t in r04tree .; do
    (cd $t && timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline $cfg > /tmp/ab.json 2>/tmp/ab.err) || { echo "$t failed"; tail -3 /tmp/ab.err; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]);print('$cfg round $r [$t]:', d['value'], d['ms_per_step'])"
  done
done
done
