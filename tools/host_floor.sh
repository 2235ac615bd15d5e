#!/bin/bash
# Host floor: bench C2 / C4 with the stub library (tools/build_stub.sh) beside the real one, same box.
set -o pipefail
mkdir -p gpurun_out
for cfg in c2 c4; do
  a=""; [ $cfg = c4 ] && a="--config c4"
  FDDM_HIP_LIB=$GRAFT_REPO_ROOT/vlib/stub.so timeout -k 10 300 python -u bench.py $a --no-cpu-baseline > gpurun_out/hf_stub_$cfg.json 2> gpurun_out/hf_stub_$cfg.err || { echo stub $cfg failed; tail -5 gpurun_out/hf_stub_$cfg.err; exit 1; }
  timeout -k 10 300 python -u bench.py $a --no-cpu-baseline > gpurun_out/hf_real_$cfg.json 2> gpurun_out/hf_real_$cfg.err || { echo real $cfg failed; tail -5 gpurun_out/hf_real_$cfg.err; exit 1; }
  for k in stub real; do
    python3 -c "import json; d=json.loads(open('gpurun_out/hf_${k}_$cfg.json').read().strip().splitlines()[-1]); print('$cfg $k', 'ms/step', d['ms_per_step'], 'host', d['host_ms_per_step'])"
  done
done
