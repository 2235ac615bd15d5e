# attn7_bench under library variants: bash tools/probe/var_bench.sh name1 name2 ... (vlib/<name>.so; "-" = in-tree)
for v in "$@"; do
  if [ "$v" = "-" ]; then lib=""; else lib="FDDM_HIP_LIB=$GRAFT_REPO_ROOT/vlib/$v.so"; fi
  echo "== $v"; env $lib timeout -k 10 120 python -u tools/attn7_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
