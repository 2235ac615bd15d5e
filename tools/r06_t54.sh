#!/bin/bash
# Round 6 final tree: counters of the keep-bit producer (tools/dmask_time.py) and of WavLM attention on fwd7 vs fwd5
# (tools/wavlm_attn_time.py runs both) -> per-kernel tables (tools/pmc_generic.sh + pmc_kernels.py)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"
bash tools/pmc_generic.sh r06m_dmask "$G1:$G2" tools/dmask_time.py > gpurun_out/r06_t54_dmask.txt 2>&1 || { tail -20 gpurun_out/r06_t54_dmask.txt; exit 1; }
cat gpurun_out/r06_t54_dmask.txt
bash tools/pmc_generic.sh r06m_wavlm "$G1:$G2" tools/wavlm_attn_time.py > gpurun_out/r06_t54_wavlm.txt 2>&1 || { tail -20 gpurun_out/r06_t54_wavlm.txt; exit 1; }
cat gpurun_out/r06_t54_wavlm.txt
