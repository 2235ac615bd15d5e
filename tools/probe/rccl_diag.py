"""Diagnose the world-1 forced-DP step: the plain step, gloo and nccl world-1 groups, and nccl without the
overlapped reducer (bulk all-reduce after backward); pairwise per-tensor relative differences of the gradients at
both steps (KL, L_fd) and of the final parameters.
  python tools/probe/rccl_diag.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "fddm-asr_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(backend, overlap, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import datetime
    import torch.distributed as dist
    from fddm_hip import dist as fdist
    import test_gpu_dist as T
    from helpers import CollectiveLog
    if backend is not None:
        kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=0, world_size=1, timeout=datetime.timedelta(seconds=120), **kw)
        fdist.force_dp(True)
        if not overlap:
            class NoRed:
                def __init__(self, arena, *a, **k):
                    pass
            fdist.OverlapReducer = NoRed
    final = {}
    with CollectiveLog() as cl:
        grads = T._c2_dp_grads(0, 1, params_out=final)
    q.put(([{n: (None if v is None else v.numpy()) for n, v in gr.items()} for gr in grads],
           {n: v.numpy() for n, v in final.items()}, len(cl.log)))
    if backend is not None:
        dist.destroy_process_group()


def run(backend, overlap=True):
    import test_gpu_dist as T
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=worker, args=(backend, overlap, T._free_port(), q))
    p.start()
    out = q.get(timeout=400)
    p.join(timeout=60)
    return out


def rel(a, b):
    a, b = torch.from_numpy(a).double(), torch.from_numpy(b).double()
    return float((a - b).norm()) / max(float(b.norm()), 1e-12)


def main():
    runs = {"plain": run(None), "gloo": run("gloo"), "nccl": run("nccl"), "nccl_bulk": run("nccl", False),
            "gloo_bulk": run("gloo", False)}
    for k, v in runs.items():
        print(k, "collectives", v[2], flush=True)
    names = list(runs)
    for i in range(len(names)):
        for j in range(i + 1, len(names)):
            a, b = runs[names[i]], runs[names[j]]
            for st in range(2):
                diffs = sorted(((rel(a[0][st][n], v), n) for n, v in b[0][st].items() if v is not None
                                and a[0][st][n] is not None), reverse=True)
                print(f"{names[i]:9s} vs {names[j]:9s} step {st}: worst {diffs[0][0]:.2e} {diffs[0][1]}; "
                      f"n>1e-6 {sum(d > 1e-6 for d, _ in diffs)}/{len(diffs)}; 5th {diffs[min(4, len(diffs)-1)]}",
                      flush=True)
            pd = sorted(((rel(a[1][n], v), n) for n, v in b[1].items()), reverse=True)
            print(f"{names[i]:9s} vs {names[j]:9s} params: worst {pd[0][0]:.2e} {pd[0][1]}", flush=True)


if __name__ == "__main__":
    main()
