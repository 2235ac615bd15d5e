"""Per-kernel averages of every counter of every pass in a tools/pmc_generic.sh output directory, plus the kernel
trace's average duration. Derived: MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8); the
SQ_WAIT*/ACTIVE* counters divided by SQ_WAVE_CYCLES (fractions of wave lifetime).
  python tools/pmc_kernels.py gpurun_out/pmcg_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(n):
    return n.replace("unsigned short", "bf16").replace("fddm::", "").replace("attn::", "")[:60]


def main():
    root = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            names[did] = r["Kernel_Name"]
            per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        for did, cs in per.items():
            for c, v in cs.items():
                vals[names[did]][c].append(v)
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(root, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    counters = sorted({c for k in vals for c in vals[k]})
    rel = [c for c in counters if c.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY_CYCLES", "SQ_INST_LEVEL"))]
    print("| kernel | us | " + " | ".join(counters) + " | MFMA busy | " + " | ".join(c + "/WAVE_CYC" for c in rel) + " |")
    print("|---" * (2 + len(counters) + 1 + len(rel)) + "|")
    for k in sorted(vals, key=lambda k: -sum(dur.get(k, [0]))):
        avg = {c: sum(v) / len(v) for c, v in vals[k].items()}
        us = sum(dur[k]) / len(dur[k]) / 1e3 if dur.get(k) else 0.0
        busy = ""
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and avg.get("GRBM_GUI_ACTIVE"):
            busy = f"{avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024.0 * avg['GRBM_GUI_ACTIVE'] / 8.0):.3f}"
        wc = avg.get("SQ_WAVE_CYCLES")
        fr = [f"{avg[c] / wc:.3f}" if (wc and c in avg) else "" for c in rel]
        print(f"| `{short(k)}` | {us:.1f} | " + " | ".join(f"{avg.get(c, float('nan')):.4g}" for c in counters) +
              f" | {busy} | " + " | ".join(fr) + " |")


if __name__ == "__main__":
    main()
