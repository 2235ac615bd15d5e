"""Where do the small fill / copy kernels of a train step come from? torch.profiler (CPU ops with Python stacks) over
STEPS train steps of bench.py's setup (CENSUS_ARGS as in tools/op_census.py); prints, per aten op among fill_ /
zero_ / copy_ / zeros / clone / to, the count per step by input shape and the innermost Python frame of this repo
(or of torch) that issued it.
   CENSUS_ARGS="--config c4" python tools/fill_sources.py [steps]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402

OPS = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::zeros", "aten::clone", "aten::_to_copy", "aten::zeros_like")


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sys.argv = [sys.argv[0], "--steps", str(steps), "--warmup", "4", "--no-cpu-baseline"] + \
        os.environ.get("CENSUS_ARGS", "").split()
    args = bench.parse()
    device = torch.device("cuda", 0)
    torch.manual_seed(1337)
    T_, cfg, models, opt = bench.build(args, device)
    from fddm_hip import runtime as rt
    rt.reseed(1337)
    enc, dec, sp, te, tp, sch = models
    batches = bench.synthetic_batches(args, device, 4, 1000)
    gs = cfg.lfd["n_step_fd"]
    gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, [batches[i % 4] for i in range(4)], opt, device, cfg, gs,
                               None, 0, False)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        T_.train_one_epoch(enc, dec, sp, te, tp, sch, [batches[i % 4] for i in range(steps)], opt, device, cfg, gs,
                           None, 1, False)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        stack = list(ev.stack or [])
        site = next((f for f in stack if ROOT in f and "fill_sources" not in f), stack[0] if stack else "?")
        site = site.replace(ROOT + "/", "")
        shapes = str(ev.input_shapes[:1]) if ev.input_shapes else ""
        cnt[(ev.name, shapes, site)] += 1
    print(f"aten fills / copies per step (over {steps} steps):")
    for (name, shp, site), n in cnt.most_common(60):
        print(f"  {n / steps:7.2f}  {name:18s} {shp[:40]:40s} {site[:110]}")


if __name__ == "__main__":
    main()
