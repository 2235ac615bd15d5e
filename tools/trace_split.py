"""Per-stream anatomy of the overlapped train step from a rocprofv3 kernel trace (run_kernel_trace.csv of
`rocprofv3 --kernel-trace -- python3 bench.py ...`): a window of N steps is delimited by the encoder's conv-0
launches (one per encoded batch, on the encoder's side stream); per stream it reports busy time (union of its
kernels' intervals) per step, the time both streams run at once, and the top kernels per stream.
  python tools/trace_split.py <run_kernel_trace.csv> [first conv0 index] [steps]"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"^void ", "", n)
    n = n.replace("fddm::", "").replace("unsigned short", "bf16")
    return n[:90]


def union(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def main():
    path = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows]
    ks.sort()
    c0 = [k for k in ks if "conv0_gram_kernel" in k[3]]   # one per encoded batch (the side stream)
    t0, t1 = c0[first][0], c0[first + n][0]
    win = [k for k in ks if t0 <= k[0] < t1]
    per = defaultdict(list)
    for a, b, s, name in win:
        per[s].append((a, b, name))
    span = (t1 - t0) / n / 1e3
    print(f"window: conv0 launches {first}..{first + n}: {n} steps, {span:.1f} us per step (wall)\n")
    print("| stream | kernels/step | busy us/step | busy share |")
    print("|---|---|---|---|")
    for s, lst in sorted(per.items(), key=lambda kv: -len(kv[1])):
        b = union([(a, e) for a, e, _ in lst]) / n / 1e3
        print(f"| {s} | {len(lst) / n:.0f} | {b:.1f} | {b / span:.2f} |")
    streams = sorted(per, key=lambda s: -len(per[s]))[:2]
    if len(streams) == 2:
        ia = [(a, e) for a, e, _ in per[streams[0]]]
        ib = [(a, e) for a, e, _ in per[streams[1]]]
        both = union(ia) + union(ib) - union(ia + ib)
        print(f"\nboth streams busy at once: {both / n / 1e3:.1f} us/step")
    for s in streams:
        tot = defaultdict(lambda: [0, 0])
        for a, e, name in per[s]:
            tot[short(name)][0] += e - a
            tot[short(name)][1] += 1
        print(f"\n### stream {s}: top kernels (us per step, launches per step)\n")
        print("| kernel | us/step | launches/step | avg us |")
        print("|---|---|---|---|")
        for name, (t, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:25]:
            print(f"| `{name}` | {t / n / 1e3:.1f} | {c / n:.1f} | {t / c / 1e3:.1f} |")


if __name__ == "__main__":
    main()
