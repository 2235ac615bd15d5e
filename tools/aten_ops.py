"""Counts the ATen ops that launch device work inside the C2 train step (bench.py's build) and where they come
from: torch.profiler over 4 steady-state steps, grouped by op name and the innermost repo source line."""
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda:0")
    T_, cfg, models, opt = bench.build(args, dev)
    enc, dec, sp, te, tp, sch = models
    batches = bench.synthetic_batches(args, dev, 4, 1000)
    gs = 4
    gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, batches, opt, dev, cfg, gs, None, 0, False)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, batches, opt, dev, cfg, gs, None, 0, False)
        torch.cuda.synchronize()
    want = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::zeros", "aten::cat", "aten::stack", "aten::clone", "aten::add",
            "aten::mul", "aten::sum", "aten::mean", "aten::index", "aten::ne", "aten::eq", "aten::to",
            "aten::contiguous", "aten::where", "aten::expand", "aten::zeros", "aten::ones", "aten::empty")
    cnt = Counter()
    for ev in prof.events():
        if ev.name not in want:
            continue
        if ev.name in ("aten::fill_", "aten::copy_") and os.environ.get("PARENTS"):
            chain, p = [], ev.cpu_parent
            while p is not None and len(chain) < 4:
                chain.append(p.name[:60])
                p = p.cpu_parent
            cnt[(ev.name, " < ".join(chain) or "(top)")] += 1
            continue
        src = "?"
        for fr in (ev.stack or []):
            if ("fddm" in fr or "bench" in fr or "train" in fr or "models" in fr) and "site-packages" not in fr \
                    and "dist-packages" not in fr:
                src = fr.split("/")[-1] if "/" in fr else fr
                break
        if src == "?" and ev.stack:
            src = "|".join(f.split("/")[-1] for f in ev.stack[:3])
        cnt[(ev.name, src)] += 1
    for (name, src), n in sorted(cnt.items(), key=lambda kv: -kv[1]):
        print(f"{n / 4:6.1f}/step  {name:18s} {src}")


if __name__ == "__main__":
    main()
