set -o pipefail
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
bash tools/pmc_generic.sh a7c4b "$G1:$G2:$G3:$G4" tools/probe/attn7_one.py c4self both > gpurun_out/pmc_a7c4b.txt 2>&1 && \
bash tools/pmc_generic.sh a7c2b "$G1:$G2:$G3:$G4" tools/probe/attn7_one.py c2self both > gpurun_out/pmc_a7c2b.txt 2>&1
rc=$?; head -12 gpurun_out/pmc_a7c4b.txt | cut -c1-200; exit $rc
