#!/bin/bash
# round-6 measurement: default bench line + kernel trace (tools/measure.sh), fwd8 PMC at C2 self / cross
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
bash tools/measure.sh r06c || exit 1
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"
bash tools/pmc_generic.sh a8v6x "$G1:$G2" tools/probe/attn7_one.py c2cross fwd auto > gpurun_out/r06_t23_pmc_cross.txt 2>&1 || exit 1
bash tools/pmc_generic.sh a8v6s "$G1:$G2" tools/probe/attn7_one.py c2self fwd auto > gpurun_out/r06_t23_pmc_self.txt 2>&1 || exit 1
echo done
