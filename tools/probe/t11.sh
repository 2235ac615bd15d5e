set -o pipefail
for v in - lnbh - lnbh; do
  if [ "$v" = "-" ]; then lib=""; else lib="FDDM_HIP_LIB=$GRAFT_REPO_ROOT/vlib/$v.so"; fi
  echo "== $v"; env $lib timeout -k 10 100 python -u tools/ln_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
