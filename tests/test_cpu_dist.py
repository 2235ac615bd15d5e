"""world_size-2 gloo test of the DP gradient exchange (fddm_hip.dist.allreduce_grads):
ranks hold different gradients; after the exchange every rank holds the mean, bucketing (forced tiny
here so several buckets flush) keeps tensor boundaries, and params whose grad is None (projectors on
non-L_fd steps, reference train.py:400-410) stay None. CPU only."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fddm_hip import dist as fdist
        shapes = [(3, 5), (7,), (2, 2, 2), (11, 3), (1,)]
        params = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
        for i, p in enumerate(params):
            if i == 3:
                continue  # grad None on every rank
            g = torch.Generator().manual_seed(100 * rank + i)
            p.grad = torch.randn(p.shape, generator=g)
        fdist.allreduce_grads(params, bucket_bytes=64)
        q.put((rank, [None if p.grad is None else p.grad.numpy().copy() for p in params]))   # by value: the worker may exit first
    finally:
        dist.destroy_process_group()


def test_allreduce_grads_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shapes = [(3, 5), (7,), (2, 2, 2), (11, 3), (1,)]
    for i, s in enumerate(shapes):
        if i == 3:
            assert got[0][i] is None and got[1][i] is None
            continue
        exp = sum(torch.randn(s, generator=torch.Generator().manual_seed(100 * r + i)) for r in range(world)) / world
        for r in range(world):
            torch.testing.assert_close(torch.from_numpy(got[r][i]), exp, rtol=1e-6, atol=1e-6)


def _overlap_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fddm_hip import dist as fdist
        from fddm_hip import runtime as rt
        shapes = [(40, 3), (7,), (2, 9, 2), (64,), (5, 5), (33,)]
        params = [torch.nn.Parameter(torch.zeros(s)) for s in shapes]
        order = [params[i] for i in (4, 1, 5, 0, 3, 2)]       # "backward" finalises them in this order
        arena = rt.GradArena(params, order)
        red = fdist.OverlapReducer(arena, bucket_bytes=256)   # tiny buckets: slices launch mid-"backward"
        inflight = []
        from helpers import CollectiveLog
        for step in range(2):
            arena.zero_()
            with CollectiveLog() as cl:
                for i, p in enumerate(order):
                    g = torch.Generator().manual_seed(1000 * step + 100 * rank + i)
                    p.grad.add_(torch.randn(p.shape, generator=g))
                    if rank == 1 and i % 2 == 0:
                        continue                   # rank 1 reports some params late (in pairs): same collectives
                    rt.grads_ready([p] if rank == 0 else order[max(0, i - 1):i + 1])
                    inflight.append(len(red.works))
                fdist.allreduce_grads(params, average=(step == 0))     # step 1: the SUM (fused AdamW applies 1/W)
            q.put((rank, step, [p.grad.numpy().copy() for p in order], max(inflight), cl.log))   # by value
    finally:
        dist.destroy_process_group()


def test_overlap_reducer_gloo_world2():
    """Arena laid out in backward order; slices all-reduced asynchronously as soon as a bucket's worth of
    slots is final (fddm_hip.dist.OverlapReducer), the tail at allreduce_grads; two steps (reset between), the
    second leaving the ranks' sum (average=False, the fused AdamW's grad_scale path). Rank 1 reports its
    gradients ready in a different grouping (late, in pairs); both ranks still issue the same collectives."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, logs = {}, {}
    for _ in range(2 * world):
        r, step, gs, nin, log = q.get(timeout=120)
        got[(r, step)] = gs
        logs[(r, step)] = log
        assert nin > 0, "no slice was in flight before allreduce_grads"
    for step in range(2):   # identical collective sequences on both ranks, although rank 1 reported grads late
        assert logs[(0, step)] == logs[(1, step)] and len(logs[(0, step)]) > 2, (logs[(0, step)], logs[(1, step)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shapes = [(40, 3), (7,), (2, 9, 2), (64,), (5, 5), (33,)]
    order_shapes = [shapes[i] for i in (4, 1, 5, 0, 3, 2)]
    for step in range(2):
        for i, s in enumerate(order_shapes):
            exp = sum(torch.randn(s, generator=torch.Generator().manual_seed(1000 * step + 100 * r + i))
                      for r in range(world)) / (world if step == 0 else 1)
            for r in range(world):
                torch.testing.assert_close(torch.from_numpy(got[(r, step)][i]), exp, rtol=1e-6, atol=1e-6)


def _bcast_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fddm_hip import dist as fdist
        torch.manual_seed(10 + rank)                 # different inits per rank
        ts = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(9)), torch.randint(0, 9, (4,))]
        v0 = ts[0]._version
        fdist.broadcast_params(ts, bucket_bytes=32)  # tiny buckets: several flushes, mixed dtypes
        q.put((rank, [t.detach().numpy().copy() for t in ts], ts[0]._version > v0))
    finally:
        dist.destroy_process_group()


def test_broadcast_params_gloo_world2():
    """DP replicas start from rank 0's weights (fddm_hip.dist.broadcast_params, called once by train_one_epoch):
    every rank ends with rank 0's values, per dtype, across bucket boundaries, and the in-place copy moves the
    version counters (so cached bf16 / permuted weight copies are rebuilt)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, vals, bumped = q.get(timeout=120)
        got[r] = (vals, bumped)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(10)
    ref = [torch.randn(5, 3), torch.randn(9), torch.randint(0, 9, (4,))]
    for r in range(world):
        assert got[r][1]
        for a, b in zip(got[r][0], ref):
            assert torch.equal(torch.from_numpy(a), b)
