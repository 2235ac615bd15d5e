"""Which torch ops does the C2 train step issue around the HIP kernels, and from where? Runs bench.py's C2 setup and
records, during STEPS steps, every torch function / tensor method call (TorchFunctionMode) made from this repo's
Python files, keyed by (op, caller file:line). Prints the calls per step, most frequent first — the fills, copies and
elementwise ops that become small GPU kernels (FillFunctor, copyBuffer, elementwise) next to the library's launches.
Autograd-internal work (grad accumulation, engine zero-fills) is not a Python call and is not listed.
   python tools/op_census.py [steps]"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402
from torch.overrides import TorchFunctionMode  # noqa: E402

import bench  # noqa: E402

SKIP = {"data_ptr", "stride", "size", "dim", "is_contiguous", "numel", "__get__", "shape", "dtype", "device",
        "element_size", "storage_offset", "requires_grad", "is_cuda", "__len__", "__repr__", "__format__", "__bool__",
        "__int__", "__index__", "__hash__", "grad", "_version", "data", "is_leaf", "register_hook", "detach",
        "view", "view_as", "reshape", "unflatten", "flatten", "t", "transpose", "permute", "__getitem__", "squeeze",
        "unsqueeze", "expand", "as_strided", "narrow", "chunk", "split", "unbind", "select", "contiguous", "nelement",
        "untyped_storage", "_base", "is_floating_point", "get_device", "new_empty", "empty", "empty_like"}


class Census(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.cnt = collections.Counter()

    def __torch_function__(self, func, types, args=(), kwargs=None):
        name = getattr(func, "__name__", str(func))
        if name not in SKIP:
            site = "?"
            for fr in reversed(traceback.extract_stack(limit=12)[:-1]):
                if fr.filename.startswith(ROOT) and "op_census" not in fr.filename:
                    site = f"{os.path.relpath(fr.filename, ROOT)}:{fr.lineno}"
                    break
            self.cnt[(name, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    sys.argv = [sys.argv[0], "--steps", str(steps), "--warmup", "4", "--no-cpu-baseline"] + \
        os.environ.get("CENSUS_ARGS", "").split()   # e.g. CENSUS_ARGS="--config c4"
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
    mode = Census()
    # the backward Functions run on the autograd engine's thread, where a TorchFunctionMode is not active: the
    # kernel-issuing torch entry points are also wrapped globally (any thread) and counted by caller
    patched = []
    for owner, name in ((torch, "zeros"), (torch, "zeros_like"), (torch, "full"), (torch, "ones"), (torch, "cat"),
                        (torch, "stack"), (torch.Tensor, "zero_"), (torch.Tensor, "fill_"), (torch.Tensor, "copy_"),
                        (torch.Tensor, "clone"), (torch.Tensor, "to"), (torch.Tensor, "float"),
                        (torch.Tensor, "contiguous"), (torch.Tensor, "add_"), (torch.Tensor, "mul_")):
        orig = getattr(owner, name)

        def wrap(*a, _o=orig, _n=name, **k):
            if not mode_active[0]:
                return _o(*a, **k)
            site = "?"
            for fr in reversed(traceback.extract_stack(limit=12)[:-1]):
                if fr.filename.startswith(ROOT) and "op_census" not in fr.filename:
                    site = f"{os.path.relpath(fr.filename, ROOT)}:{fr.lineno}"
                    break
            mode.cnt[("*" + _n, site)] += 1
            return _o(*a, **k)
        setattr(owner, name, wrap)
        patched.append((owner, name, orig))
    mode_active = [True]
    with mode:
        T_.train_one_epoch(enc, dec, sp, te, tp, sch, [batches[i % 4] for i in range(steps)], opt, device, cfg, gs,
                           None, 1, False)
    torch.cuda.synchronize()
    mode_active[0] = False
    for owner, name, orig in patched:
        setattr(owner, name, orig)
    print(f"torch calls per step from this repo (over {steps} steps):")
    print("(* = counted by the global wrappers, any thread; a call on the main thread may be counted twice)")
    for (name, site), n in mode.cnt.most_common(90):
        print(f"  {n / steps:7.2f}  {name:32s} {site}")


if __name__ == "__main__":
    main()
