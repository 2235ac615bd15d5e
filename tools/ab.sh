#!/bin/bash
# bench.py A/B on ONE box (DVFS and box-to-box spread make cross-box comparisons meaningless): every argument is one
# arm — a space-separated list of VAR=value settings, or "-" for the defaults — and the arms run alternating for
# ROUNDS rounds (default 2). Replaces the round-2 one-offs (ab_env*.sh, cap_sweep*.sh, deccap/ncu/splitk sweeps):
#   encoder CU caps:       bash tools/ab.sh "FDDM_ENC_CUS_CONV=128 FDDM_ENC_CUS=192" "FDDM_ENC_CUS_CONV=144 FDDM_ENC_CUS=192"
#   graph replay:          bash tools/ab.sh - "FDDM_STEP_GRAPH=1"
#   extra bench.py flags:  BENCH_ARGS="--config c4" ROUNDS=3 bash tools/ab.sh - "FDDM_ENC_CUS=208"
rounds=${ROUNDS:-2}
args=${BENCH_ARGS:-}
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
  i=0
  for arm in "$@"; do
    i=$((i+1))
    envs=$arm
    [ "$arm" = "-" ] && envs=""
    out=gpurun_out/ab_${i}_r$r
    env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline $args > $out.json 2> $out.err || exit 1
    python3 -c "import json;d=json.loads(open('$out.json').read().strip().splitlines()[-1]);print('round $r [$arm]:', d['value'], d['unit'], d['ms_per_step'], 'ms')"
  done
done
