mkdir -p gpurun_out/pmc2
for v in base variants/lib_gm1.so variants/lib_gm8.so variants/lib_nopersist.so variants/lib_nopersist_gm1.so; do
  if [ $v = base ]; then L=$PWD/fddm-asr_amd/fddm_hip/libfddm_hip.so; else L=$PWD/$v; fi
  FDDM_HIP_LIB=$L timeout -k 5 120 python tools/g256_sweep.py || exit 1
done > gpurun_out/sweep2.log 2>&1
cd /tmp; export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for v in base gm1 nopersist_gm1; do
  if [ $v = base ]; then L=$PWD/fddm-asr_amd/fddm_hip/libfddm_hip.so; else L=$PWD/variants/lib_$v.so; fi
  FDDM_HIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc2/$v -o p -- python3 tools/g256_one.py 8192 8192 8192 > gpurun_out/pmc2/$v.log 2>&1 || exit 1
  FDDM_HIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc2/${v}_ff1 -o p -- python3 tools/g256_one.py 15968 3072 768 > gpurun_out/pmc2/${v}_ff1.log 2>&1 || exit 1
done
