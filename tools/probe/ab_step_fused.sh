# Same-box A/B of the whole train step: this library against vlib/base.so (the round-5 library before the fused
# attention backward), alternating default bench runs (C2), then C4
set -o pipefail
for cfg in "" "--config c4"; do
for r in 1 2 3; do
  for lib in vlib/base.so fddm-asr_amd/fddm_hip/libfddm_hip.so; do
    FDDM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline $cfg > /tmp/ab.json 2>/tmp/ab.err || { echo "$lib failed"; tail -3 /tmp/ab.err; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]);print('$cfg round $r [$lib]:', d['value'], d['ms_per_step'])"
  done
done
done
