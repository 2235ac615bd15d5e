#!/bin/bash
# fused KL alone: counters (waits, VALU, occupancy, bytes)
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PWD/fddm-asr_amd:$PWD/tests
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES"
G2="FETCH_SIZE"
G3="WRITE_SIZE"
G4="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU GRBM_GUI_ACTIVE"
bash tools/pmc_generic.sh kl "$G1:$G2:$G3:$G4" tools/kl_time.py > gpurun_out/r06_t30_kl.txt 2>&1 || exit 1
echo done
