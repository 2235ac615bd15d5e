#!/bin/bash
# decoder step alone on the whole chip (condition precomputed): phase timeline
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 200 python -u tools/timeline.py --dec-only > gpurun_out/r06b_timeline_deconly.txt 2>&1 || exit 1
echo done
