set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tr7
for s in c2self c2cross c4self c4cross; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr7/$s -o run -- python3 tools/probe/attn7_one.py $s both > gpurun_out/tr7/$s.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
for s in ("c2self", "c2cross", "c4self", "c4cross"):
    d = defaultdict(list)
    for f in glob.glob(f"gpurun_out/tr7/{s}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "attn" in n or "fwd" in n or "dq" in n or "dkv" in n or "bwd" in n:
                d[n.split("(")[0].replace("void ", "").replace("fddm::attn::", "")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(s, "  ".join(f"{k} {sum(v)/len(v):.1f}us x{len(v)}" for k, v in sorted(d.items())))
PY
