"""Data-parallel gradient exchange: one process per GPU, torch.distributed over
RCCL (backend "nccl" on ROCm) / gloo on CPU. The train step's only collective is the gradient
all-reduce; grads are packed into ~64 MB flat buckets so each RCCL call moves large messages over
xGMI, then averaged. Parameters whose grad is None (projectors on non-L_fd steps) are skipped on
every rank alike, since all ranks share global_step."""
from __future__ import annotations

import torch
import torch.distributed as dist

BUCKET_BYTES = 64 << 20


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


@torch.no_grad()
def allreduce_grads(params, bucket_bytes: int = BUCKET_BYTES) -> None:
    W = world()
    if W <= 1:
        return
    params = list(params)
    arena = next((a for a in (getattr(p, "_fddm_arena", None) for p in params) if a is not None), None)
    if arena is not None and all(p.grad is not None and p.grad.data_ptr() == v.data_ptr()
                                 for p, v in zip(arena.params, arena.views)):
        # the arena is already flat: all-reduce it in place in bucket-sized slices
        flat = arena.flat
        step = max(1, bucket_bytes // 4)
        for s0 in range(0, flat.numel(), step):
            sl = flat[s0:s0 + step]
            dist.all_reduce(sl, op=dist.ReduceOp.SUM)
            sl.mul_(1.0 / W)
        inside = set(id(p) for p in arena.params)
        params = [p for p in params if id(p) not in inside]
    grads = [p.grad for p in params if p.grad is not None]
    bucket, size = [], 0

    def flush(bk):
        if not bk:
            return
        flat = torch.cat([g.reshape(-1) for g in bk])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        flat.mul_(1.0 / W)
        off = 0
        for g in bk:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    for g in grads:
        bucket.append(g)
        size += g.numel() * g.element_size()
        if size >= bucket_bytes:
            flush(bucket)
            bucket, size = [], 0
    flush(bucket)
