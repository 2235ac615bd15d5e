"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    n = r["Name"].replace("unsigned short", "bf16").replace("fddm::", "")
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {100*float(r['TotalDurationNs'])/tot:5.1f}% calls {r['Calls']:>5} "
          f"avg {float(r['AverageNs'])/1e3:9.1f} us  {n[:120]}")
print("total ms", round(tot / 1e6, 2))
