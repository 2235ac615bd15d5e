"""DP gradient exchange overlapped with the decoder backward, on the GPU (fddm_hip.dist.OverlapReducer):
two ranks on cuda:0 (gloo moves the CUDA slices; RCCL on a multi-GPU node runs the same call sequence) each
run the decoder fwd + KL + backward on half of a batch with tiny buckets, so arena slices are all-reduced
while later blocks' backward kernels still accumulate. The averaged arena must equal the gradient of one
process on the whole batch (the KL loss is a batch mean; dropout 0; fp32 parity mode)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

V, d, H, NL, FF, S, L, T_STEPS = 1000, 128, 2, 3, 256, 24, 16, 10


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch():
    g = torch.Generator().manual_seed(11)
    B = 4
    x0 = torch.randint(1, V, (B, L), generator=g)
    x0[1, 12:] = 0
    x0[3, 9:] = 0
    xt = torch.randint(1, V, (B, L), generator=g)
    xt[x0 == 0] = 0
    t = torch.tensor([1, 4, 7, 10])
    cond = torch.randn(B, S, d, generator=g)
    return x0, xt, t, cond


def _grads(rank, world, bucket_bytes):
    import train as T_
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from fddm_hip import dist as fdist
    from fddm_hip import runtime as rt
    from fddm_hip.optim import FusedAdamW
    from test_gpu_models import make_decoder
    dev = torch.device("cuda:0")
    x0, xt, t, cond = _batch()
    sl = slice(None) if world == 1 else slice(2 * rank, 2 * rank + 2)
    x0, xt, t, cond = (v[sl].to(dev) for v in (x0, xt, t, cond))
    with rt.use_precision("fp32"):
        dec = make_decoder(V, d, H, NL, FF)
        dec.train()
        opt = FusedAdamW(list(dec.parameters()))
        opt.use_grad_arena(list(dec.parameters()), dec.grad_ready_order())
        red = fdist.OverlapReducer(opt.arena, bucket_bytes=bucket_bytes) if world > 1 else None
        sch = T_.SchedulerAdapter(DiscreteDiffusionScheduler(K=V, T=T_STEPS, device=dev))
        opt.zero_grad()
        logits = dec(xt, t, cond, x_mask=x0 != 0)
        loss = sch.kl_term(xt, x0, logits, t, x0 != 0)
        loss.backward()
        inflight = 0 if red is None else len(red.works)
        fdist.allreduce_grads(list(dec.parameters()))
        torch.cuda.synchronize()
    return {n: p.grad.detach().cpu().clone() for n, p in dec.named_parameters()}, inflight


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        gr, nin = _grads(rank, world, 64 << 10)
        q.put((rank, {n: v.numpy() for n, v in gr.items()}, nin))   # by value: the worker exits first
    finally:
        dist.destroy_process_group()


def test_overlapped_allreduce_matches_full_batch_gradient():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, gr, nin = q.get(timeout=100)
        got[r] = (gr, nin)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref, _ = _grads(0, 1, 0)
    assert got[0][1] > 1, "expected several slices in flight before backward finished"
    for n, g in ref.items():
        scale = g.abs().max().item() + 1e-12
        for r in range(world):
            err = (torch.from_numpy(got[r][0][n]) - g).abs().max().item() / scale
            assert err < 1e-4, f"{n} rank {r}: rel err {err:.2e}"
