"""Per-layer rows of the WavLM conv feature extractor from a rocprofv3 kernel trace (run_kernel_trace.csv of
`rocprofv3 --kernel-trace -- python3 bench.py ...`). The conv layers 1-6 all run as `gemm256_kernel<3, bf16, true>`
(persistent grid: the grid is the CU cap x 512, not the layer), so a layer is identified by its position: conv layer
k is the k-th such launch after each `conv0_mfma_kernel` launch on the same stream. Writes one JSON with, per layer,
avg / min / max / count of the launch duration, split by grid (the in-step launches run on the conv cap, the one
untimed `roofline_isolated` step on the whole chip), the algorithmic FLOPs per launch at the trace's batch, and the
kernel-source hash the bench keys its PMC traffic file on.
  python tools/conv_rows.py <run_kernel_trace.csv> <out.json> [batch] [seconds]"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def layer_flops(batch, seconds):
    n = int(16000 * seconds)
    out = []
    for i, (k, st) in enumerate(zip((10, 3, 3, 3, 3, 2, 2), (5, 2, 2, 2, 2, 2, 2))):
        n = (n - k) // st + 1
        if i:
            out.append(2.0 * batch * n * 512 * k * 512)
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    seconds = float(sys.argv[4]) if len(sys.argv) > 4 else 10.0
    rows = list(csv.DictReader(open(src)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    pos = {}            # stream -> index of the next conv layer after the last conv0 on it
    per = defaultdict(list)
    for r in rows:
        name, st = r["Kernel_Name"], r["Stream_Id"]
        if "conv0_mfma_kernel" in name:
            pos[st] = 1
        elif "gemm256_kernel<3," in name and st in pos and pos[st] <= 6:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per[(pos[st], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))].append(dur)
            pos[st] += 1
    fl = layer_flops(batch, seconds)
    import bench
    out = {"source": os.path.relpath(src, ROOT), "recipe": "tools/conv_rows.py over tools/measure.sh's kernel trace",
           "batch": batch, "kernel_src_sha": bench.conv1_src_sha(), "layers": []}
    for (layer, wgs), v in sorted(per.items()):
        avg = sum(v) / len(v)
        out["layers"].append({"layer": layer, "workgroups": wgs, "launches": len(v), "avg_us": round(avg, 1),
                              "min_us": round(min(v), 1), "max_us": round(max(v), 1),
                              "gflop_per_launch": round(fl[layer - 1] / 1e9, 2),
                              "tflops_avg": round(fl[layer - 1] / (avg * 1e-6) / 1e12, 1),
                              "frac_of_2500": round(fl[layer - 1] / (avg * 1e-6) / 2.5e15, 4)})
    json.dump(out, open(dst, "w"), indent=1)
    for l_ in out["layers"]:
        print(l_)


if __name__ == "__main__":
    main()
