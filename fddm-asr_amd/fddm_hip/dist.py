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
