# counters of the fused attention backward (bwdf7) next to the split pair (dq7 + dkv7) at the C2 self / cross shapes
set -o pipefail
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
bash tools/pmc_generic.sh bfc2s "$G1:$G2:$G3:$G4" tools/probe/attn7_one.py c2self bwd nofused,auto > gpurun_out/pmc_bfc2s.txt 2>&1 && \
bash tools/pmc_generic.sh bfc2c "$G1:$G2:$G3:$G4" tools/probe/attn7_one.py c2cross bwd nofused,auto > gpurun_out/pmc_bfc2c.txt 2>&1
rc=$?; grep "bwdf7\|dq7\|dkv7" gpurun_out/pmc_bfc2s.txt gpurun_out/pmc_bfc2c.txt | cut -c1-160; exit $rc
