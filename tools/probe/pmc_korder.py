"""FETCH_SIZE of the longest gemm256_kernel<3 dispatch per grid size (conv layer 1 at caps 128 / 256) from a
rocprofv3 --pmc FETCH_SIZE run of tools/conv_bench.py: bytes = 2 * FETCH_SIZE KB (gfx950 correction, tools/pmc_traffic.py).
  python tools/probe/pmc_korder.py <run_counter_collection.csv>"""
import csv, sys
from collections import defaultdict
rows = defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    if r.get("Counter_Name") != "FETCH_SIZE" or "gemm256_kernel<3" not in r.get("Kernel_Name", ""):
        continue
    d = r.get("Dispatch_Id") or r.get("Correlation_Id")
    rows[d]["grid"] = int(float(r.get("Grid_Size", 0) or 0))
    rows[d]["dur"] = int(r.get("End_Timestamp", 0)) - int(r.get("Start_Timestamp", 0))
    rows[d]["v"] = rows[d].get("v", 0.0) + float(r.get("Counter_Value", 0) or 0)
best = {}
for d, x in rows.items():
    g = x["grid"]
    if g not in best or x["dur"] > best[g]["dur"]:
        best[g] = x
for g, x in sorted(best.items()):
    print(f"grid {g}: longest dispatch {x['dur'] / 1e3:.1f} us, fetched {2 * x['v'] * 1024 / 1e9:.3f} GB")
