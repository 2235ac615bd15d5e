#!/bin/bash
# LN backward slab height: 16 / 32 / 64 rows per workgroup (timing-only variants, tools/build_variant.sh)
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
for v in base ln16 ln64 base; do
  if [ $v = base ]; then unset FDDM_HIP_LIB; else export FDDM_HIP_LIB=$PWD/abl/$v.so; fi
  echo "== $v" >> gpurun_out/r06_t17_ln.txt
  timeout -k 10 120 python -u tools/ln_bench.py >> gpurun_out/r06_t17_ln.txt 2>&1 || exit 1
done
echo done
