set -o pipefail
for v in - dkv3 - dkv3; do
  if [ "$v" = "-" ]; then lib=""; else lib="FDDM_HIP_LIB=$GRAFT_REPO_ROOT/vlib/$v.so"; fi
  echo "== $v"; env $lib timeout -k 10 200 python -u tools/attn7_bench.py 50 2>&1 | grep -v amdgpu.ids | sed 's/v6:.*| auto/auto/' || exit 1
done
