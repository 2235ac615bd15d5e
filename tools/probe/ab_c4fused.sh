# C4 step with the fused attention backward taken up to Lq 1024 (vlib/fq1024.so: C4's 512-query shapes, 192
# workgroups of 16 tile-steps, the CUs it leaves idle free for the other stream) against the default (pair at C4)
set -o pipefail
for r in 1 2 3; do
  for lib in fddm-asr_amd/fddm_hip/libfddm_hip.so vlib/fq1024.so; do
    FDDM_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --config c4 --steps 20 --warmup 4 --no-cpu-baseline > /tmp/ab.json 2>/tmp/ab.err || { echo "$lib failed"; tail -3 /tmp/ab.err; exit 1; }
    python3 -c "import json;d=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]);print('c4 round $r [$lib]:', d['value'], d['ms_per_step'])"
  done
done
