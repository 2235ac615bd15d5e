#!/bin/bash
# fwd8 ablations (timing only) + stamps
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,auto > gpurun_out/r06_t7_bench.log 2>&1 || exit 1
for v in nodrop norowsum noexp nowait; do
  FDDM_HIP_LIB=$PWD/abl/$v.so timeout -k 10 120 python -u tools/attn7_bench.py 20 auto > gpurun_out/r06_t7_bench_$v.log 2>&1 || exit 1
done
FDDM_HIP_LIB=$PWD/abl/a8st.so timeout -k 10 120 python -u tools/probe/a8_stamps.py > gpurun_out/r06_t7_stamps.log 2>&1 || exit 1
echo done
