#!/bin/bash
# fwd8 diagnostics: PMC passes (fwd8 vs fwd7, C2 cross / self forward), ablation timings (no mid-tile wait, no exp)
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"
bash tools/pmc_generic.sh a8c2x "$G1:$G2" tools/probe/attn7_one.py c2cross fwd fwd7,auto > gpurun_out/r06_t5_pmc_c2x.txt 2>&1 || exit 1
bash tools/pmc_generic.sh a8c2s "$G1:$G2" tools/probe/attn7_one.py c2self fwd fwd7,auto > gpurun_out/r06_t5_pmc_c2s.txt 2>&1 || exit 1
for v in nowait noexp; do
  FDDM_HIP_LIB=$PWD/abl/$v.so timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,auto > gpurun_out/r06_t5_bench_$v.log 2>&1 || exit 1
done
echo done
FDDM_HIP_LIB=$PWD/abl/a8st.so timeout -k 10 120 python -u tools/probe/a8_stamps.py > gpurun_out/r06_t5_stamps.log 2>&1 || exit 1
echo done2
