"""Data-parallel gradient exchange: one process per GPU, torch.distributed over
RCCL (backend "nccl" on ROCm) / gloo on CPU. The train step's only collective is the gradient
all-reduce; grads are packed into ~64 MB flat buckets so each RCCL call moves large messages over
xGMI, then averaged. Parameters whose grad is None (projectors on non-L_fd steps) are skipped on
every rank alike, since all ranks share global_step."""
from __future__ import annotations

import torch
import torch.distributed as dist

BUCKET_BYTES = 64 << 20
OVERLAP_BUCKET_BYTES = 16 << 20


class OverlapReducer:
    """Gradient all-reduce overlapped with backward (BASELINE configs[2]: "grad all-reduce overlap").

    The grad arena's slots are laid out in the order backward finalises them (runtime.GradArena `order`:
    head, last decoder block, ..., first block, then FiLM / embeddings / time MLP). Backward Functions call
    runtime.grads_ready(params) once they have enqueued everything that accumulates into those slots; the
    reducer then tracks the finished prefix of the arena and, whenever it has grown by a bucket, enqueues an
    async all-reduce of that slice. RCCL orders the collective after the kernels already on the compute
    stream and runs it on its own stream, so it proceeds under the remaining blocks' backward. `finish()`
    (from allreduce_grads, after backward) launches the tail, makes the compute stream wait for every slice
    and averages. Slices are cut at fixed multiples of the bucket (not at the prefix's growth points), so the
    collective sequence is the same on every rank whatever grouping the ranks' grads_ready calls came in
    (tests/test_cpu_dist.py::test_overlap_reducer_gloo_world2 records and compares it)."""

    def __init__(self, arena, bucket_bytes: int = OVERLAP_BUCKET_BYTES):
        self.arena = arena
        self.bucket = max(1, bucket_bytes // 4)
        self.W = world()
        self.reset()
        arena.on_ready = self.on_ready
        arena.reducer = self

    def reset(self):
        self.ready = [False] * len(self.arena.params)
        self.next = 0
        self.launched = 0
        self.works = []

    def on_ready(self, params):
        a = self.arena
        for p in params:
            i = a.slot.get(id(p))
            if i is not None:
                self.ready[i] = True
        while self.next < len(self.ready) and self.ready[self.next]:
            self.next += 1
        hi = a.offs[self.next]
        while hi - self.launched >= self.bucket:      # fixed bucket-sized slices: the cut points do not depend
            self._launch(self.launched + self.bucket)  # on how each rank grouped its grads_ready calls

    def _launch(self, hi):
        lo = self.launched
        if hi <= lo:
            return
        sl = self.arena.flat[lo:hi]
        self.works.append((dist.all_reduce(sl, op=dist.ReduceOp.SUM, async_op=True), sl))
        self.launched = hi

    def finish(self, average: bool = True):
        """Launch the tail slices and make the compute stream wait for every slice. average=False leaves the
        ranks' SUM in the arena (the fused AdamW folds 1/W into its read, FusedAdamW.clip_and_step(grad_scale))."""
        n = self.arena.offs[-1]
        while self.launched < n:
            self._launch(min(n, self.launched + self.bucket))
        for w, sl in self.works:
            w.wait()
            if average:
                sl.mul_(1.0 / self.W)
        self.reset()


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


_FORCE_DP = False


def force_dp(on: bool) -> bool:
    """Tests only: run the DP exchange (rank-0 broadcast, overlapped all-reduce, global-batch L_fd statistics) even in
    a world-size-1 process group, so the collective path (e.g. RCCL's) executes on a one-GPU box. Returns the previous
    setting."""
    global _FORCE_DP
    old, _FORCE_DP = _FORCE_DP, bool(on)
    return old


def dp_active() -> bool:
    """True when the train step exchanges gradients: more than one rank, or a forced world-size-1 group."""
    return world() > 1 or (_FORCE_DP and dist.is_available() and dist.is_initialized())


def default_group():
    return dist.group.WORLD


@torch.no_grad()
def global_mean(x: torch.Tensor, group=None) -> torch.Tensor:
    """Mean over ranks of a per-rank batch mean (equal local batches): w_t's batch mean (train.py:390) of the
    global batch under DP."""
    y = x.detach().float().reshape(1).clone()
    dist.all_reduce(y, group=group)
    return (y / dist.get_world_size(group)).reshape(x.shape)


@torch.no_grad()
def broadcast_params(tensors, src: int = 0, bucket_bytes: int = BUCKET_BYTES) -> None:
    """Make every rank's copy of `tensors` (parameters / buffers) equal to rank `src`'s, in flat buckets per dtype
    (what DistributedDataParallel's constructor does): replicas that start from different random inits would
    otherwise drift apart under the averaged gradients. The copies back go through Tensor.copy_ so each tensor's
    version counter moves and every cached low-precision / permuted copy of it is rebuilt."""
    if not dp_active():
        return
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (dt, dev), ts in by_dtype.items():
        bucket, size = [], 0
        for t in ts + [None]:
            if t is not None:
                bucket.append(t)
                size += t.numel() * t.element_size()
            if bucket and (t is None or size >= bucket_bytes):
                flat = torch.cat([x.detach().reshape(-1) for x in bucket])
                dist.broadcast(flat, src=src)
                off = 0
                for x in bucket:
                    n = x.numel()
                    x.copy_(flat[off:off + n].view_as(x))
                    off += n
                bucket, size = [], 0


@torch.no_grad()
def allreduce_grads(params, bucket_bytes: int = BUCKET_BYTES, average: bool = True) -> None:
    """All-reduce the gradients of `params` over the ranks. average=True leaves the mean (torch DDP semantics);
    average=False leaves the SUM, for a consumer that applies 1/W itself (the fused AdamW's grad_scale), which saves
    a pass over every gradient."""
    W = world()
    if not dp_active():
        return
    params = list(params)
    arena = next((a for a in (getattr(p, "_fddm_arena", None) for p in params) if a is not None), None)
    if arena is not None and getattr(arena, "reducer", None) is not None:
        arena.reducer.finish(average)     # slices already in flight since backward; launch the tail, wait
        inside = set(id(p) for p in arena.params)
        params = [p for p in params if id(p) not in inside]
    elif arena is not None and all(p.grad is not None and p.grad.data_ptr() == v.data_ptr()
                                   for p, v in zip(arena.params, arena.views)):
        # the arena is already flat: all-reduce it in place in bucket-sized slices
        flat = arena.flat
        step = max(1, bucket_bytes // 4)
        for s0 in range(0, flat.numel(), step):
            sl = flat[s0:s0 + step]
            dist.all_reduce(sl, op=dist.ReduceOp.SUM)
            if average:
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
        if average:
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
