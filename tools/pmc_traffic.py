"""HBM traffic per launch of the bench's dominant kernel from two rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; MI355X_MICROARCH.md 'rocprofv3 PMC slots').

FETCH_SIZE is in KB and, on gfx950, reports half the bytes of wide coalesced streaming reads
(MI355X_MICROARCH.md § HBM): traffic = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes).
The dominant launch (WavLM conv layer 1) shares its kernel symbol with conv layers 2-6 (and the persistent
kernel's grid is one workgroup per CU for all of them); it is the dispatch of that symbol that runs longest.

  python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <kernel substring> <out.json> <batch>
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import conv1_src_sha  # noqa: E402


def load(path, counter):
    rows = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        rows[did]["name"] = r.get("Kernel_Name", "")
        rows[did]["grid"] = int(float(r.get("Grid_Size", 0) or 0))
        try:
            rows[did]["dur"] = int(r.get("End_Timestamp", 0)) - int(r.get("Start_Timestamp", 0))
        except ValueError:
            rows[did]["dur"] = 0
        rows[did][counter] = rows[did].get(counter, 0.0) + float(r["Counter_Value"])
    return rows


def pick(rows, sub, counter):
    sel = [v for v in rows.values() if sub in v["name"] and counter in v]
    if not sel:
        return None, 0, 0
    # the longest dispatches of the symbol (within 20 % of the longest): conv layer 1, once per step
    dmax = max(v.get("dur", 0) for v in sel)
    pick_ = [v for v in sel if v.get("dur", 0) >= 0.8 * dmax] if dmax > 0 else sel
    vals = [v[counter] for v in pick_]
    return sum(vals) / len(vals), len(vals), pick_[0]["grid"]


def main():
    fpath, wpath, sub, out = sys.argv[1:5]
    f, nf, g1 = pick(load(fpath, "FETCH_SIZE"), sub, "FETCH_SIZE")
    w, nw, g2 = pick(load(wpath, "WRITE_SIZE"), sub, "WRITE_SIZE")
    res = {"batch": int(sys.argv[5]) if len(sys.argv) > 5 else None, "kernel_substring": sub, "grid": g1,
           "launches": [nf, nw], "fetch_size_kb": f, "write_size_kb": w, "kernel_src_sha": conv1_src_sha(),
           "recipe": "bash tools/pmc_conv1.sh <out.json> (two rocprofv3 --pmc passes over bench.py --steps 2)"}
    if f is not None and w is not None:
        res["traffic_bytes"] = (2.0 * f + w) * 1024.0
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
