#!/bin/bash
# fwd8 with 512 registers (accumulators in AGPRs): timing + stamps; PMC of the default build (C2 cross)
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
FDDM_HIP_LIB=$PWD/abl/w1.so timeout -k 10 120 python -u tools/attn7_bench.py 20 fwd7,auto > gpurun_out/r06_t10_bench_w1.log 2>&1 || exit 1
FDDM_HIP_LIB=$PWD/abl/w1st.so timeout -k 10 120 python -u tools/probe/a8_stamps.py > gpurun_out/r06_t10_stamps_w1.log 2>&1 || exit 1
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"
G3="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
bash tools/pmc_generic.sh a8v4 "$G1:$G2:$G3" tools/probe/attn7_one.py c2cross fwd auto > gpurun_out/r06_t10_pmc.txt 2>&1 || exit 1
echo done
