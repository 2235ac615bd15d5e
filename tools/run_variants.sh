# A/B the library variants under variants/ (timing-only builds) against the in-tree library, same box
for v in fddm-asr_amd/fddm_hip/libfddm_hip.so variants/*.so; do
  FDDM_HIP_LIB=$PWD/$v timeout -k 5 120 python tools/g256_sweep.py || exit 1
done > gpurun_out/sweep3.log 2>&1
