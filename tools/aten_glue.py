"""Which ATen ops (fills, copies, cats, elementwise) still run inside the C2 train step, and from where: torch.profiler
over 4 steps of bench.py's build, grouped by op name and the innermost repository frame of the Python stack.
  python tools/aten_glue.py"""
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

sys.argv = ["bench.py"]
args = bench.parse()
dev = torch.device("cuda:0")
torch.manual_seed(1337)
T_, cfg, models, opt = bench.build(args, dev)
enc, dec, sp, te, tp, sch = models
batches = bench.synthetic_batches(args, dev, 4, 1000)
gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, batches, opt, dev, cfg, 1, None, 0, False)
torch.cuda.synchronize()
import traceback  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

SKIP = ("aten::empty", "aten::empty_strided", "aten::view", "aten::reshape", "aten::as_strided", "aten::slice",
        "aten::select", "aten::detach", "aten::t", "aten::transpose", "aten::expand", "aten::_unsafe_view",
        "aten::unflatten", "aten::alias", "aten::result_type", "aten::lift_fresh", "aten::is_nonzero", "aten::item",
        "aten::_local_scalar_dense", "aten::unbind")
cnt = Counter()


class Glue(TorchDispatchMode):
    """every ATen op dispatched inside the step, keyed by the innermost repository frame of the Python stack"""

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        n = "aten::" + func.__name__.split(".")[0]
        if n not in SKIP:
            where = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if fr.filename.startswith(ROOT) and "aten_glue" not in fr.filename:
                    where = f"{fr.filename[len(ROOT) + 1:]}:{fr.lineno}"
                    break
            cnt[(n, where)] += 1
        return func(*args, **(kwargs or {}))


with Glue():
    T_.train_one_epoch(enc, dec, sp, te, tp, sch, batches, opt, dev, cfg, gs, None, 0, False)
    torch.cuda.synchronize()
print("count per step | op | innermost repository frame")
for (n, w), c in sorted(cnt.items(), key=lambda kv: -kv[1]):
    print(f"{c / 4:6.1f} {n:32s} {w}")
