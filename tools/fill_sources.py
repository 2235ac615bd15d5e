"""Diagnostic: which Python call sites of the C2 train step launch ATen fill / copy / cast kernels. Wraps the
torch entry points that enqueue such kernels, counts calls per (op, caller file:line) over 4 steady steps, and
prints the per-step counts (same build and batches as bench.py)."""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

CNT = collections.Counter()
ON = [False]


def site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        f = fr.filename
        if ("fddm-asr_amd" in f or f.endswith("bench.py")) and "fill_sources" not in f:
            return f"{os.path.basename(f)}:{fr.lineno}"
    return "?"


def wrap(owner, name, label, pred=None):
    orig = getattr(owner, name)

    def w(*a, **k):
        if ON[0] and (pred is None or pred(a, k)):
            CNT[(label, site())] += 1
        return orig(*a, **k)
    setattr(owner, name, w)


def on_gpu(a, k):
    t = a[0] if a and isinstance(a[0], torch.Tensor) else None
    return t is None or t.is_cuda


def dev_kw(a, k):
    d = k.get("device")
    return d is not None and "cuda" in str(d)


def main():
    args = bench.parse()
    dev = torch.device("cuda:0")
    T_, cfg, models, opt = bench.build(args, dev)
    enc, dec, sp, te, tp, sch = models
    batches = bench.synthetic_batches(args, dev, 4, 1000)
    for nm in ("zeros", "ones", "full"):
        wrap(torch, nm, "torch." + nm, dev_kw)
    for nm in ("zeros_like", "ones_like", "full_like"):
        wrap(torch, nm, "torch." + nm, on_gpu)
    wrap(torch, "cat", "torch.cat")
    wrap(torch, "stack", "torch.stack")
    for nm in ("zero_", "fill_", "copy_", "clone", "contiguous", "float", "to", "repeat", "masked_fill", "sum", "mean"):
        wrap(torch.Tensor, nm, "Tensor." + nm, on_gpu)
    gs = 4
    gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, batches, opt, dev, cfg, gs, None, 0, False)
    torch.cuda.synchronize()
    ON[0] = True
    gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, batches, opt, dev, cfg, gs, None, 0, False)
    torch.cuda.synchronize()
    ON[0] = False
    for (label, s), n in sorted(CNT.items(), key=lambda kv: -kv[1]):
        print(f"{n / 4:6.2f}/step  {label:22s} {s}")


if __name__ == "__main__":
    main()
