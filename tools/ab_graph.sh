#!/bin/bash
# HIP-graph replay of the decoder step vs eager (train.StepGraphs), under the HIP runtime's graph knobs (one box,
# one round each): prints ms/step and host ms/step per arm. (DEBUG_HIP_FORCE_GRAPH_QUEUES=0 killed bench.py with
# SIGFPE in round 4, inside the HIP runtime; train._step_graph_ok refuses that setting, and the arm is gone.)
ROUNDS=1 bash tools/ab.sh - "FDDM_STEP_GRAPH=1" "FDDM_STEP_GRAPH=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" \
  "FDDM_STEP_GRAPH=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "FDDM_STEP_GRAPH=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1" > gpurun_out/ab_g.log 2>&1; cat gpurun_out/ab_g.log
for i in 1 2 3 4 5; do python3 -c "import json;d=json.loads(open('gpurun_out/ab_${i}_r1.json').read().strip().splitlines()[-1]);print($i, d['ms_per_step'], d['host_ms_per_step'])"; done
