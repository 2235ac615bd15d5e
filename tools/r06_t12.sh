#!/bin/bash
# round-6 tree at C2: bench line, kernel trace, phase timeline
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
bash tools/measure.sh r06a || exit 1
timeout -k 10 200 python -u tools/timeline.py > gpurun_out/r06a_timeline.txt 2>&1 || exit 1
echo done
