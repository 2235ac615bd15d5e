set -o pipefail
for v in - lnrw2 lnrw4 - lnrw2; do
  if [ "$v" = "-" ]; then lib=""; else lib="FDDM_HIP_LIB=$GRAFT_REPO_ROOT/vlib/$v.so"; fi
  echo "== $v"; env $lib timeout -k 10 100 python -u tools/ln_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/probe/var_fwd.sh - a7w4 - a7w4
