for v in "$@"; do
  if [ "$v" = "-" ]; then lib=""; else lib="FDDM_HIP_LIB=$GRAFT_REPO_ROOT/vlib/$v.so"; fi
  echo "== $v: $(env $lib timeout -k 10 120 python -u tools/probe/attn7_fwdonly.py 2>&1 | grep -v amdgpu.ids)" || exit 1
done
