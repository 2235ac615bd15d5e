"""Runtime state shared by the modules: compute precision, cached low-precision weight copies,
dropout seeds, and small per-shape tables (RoPE cos/sin, WavLM relative-position bias).

Precision modes (SURVEY §7 "Two precision modes"):
  * "bf16" (default on GPU): MFMA bf16 with fp32 accumulation; residual stream, LayerNorm, softmax,
    KL and L_fd statistics in fp32; fp32 master weights + AdamW.
  * "fp32": every kernel in exact fp32 (f32-input MFMA) — the parity mode checked against the oracle.
"""
from __future__ import annotations

import contextlib
import math
import os

import weakref

import torch

from . import ops

_precision = os.environ.get("FDDM_PRECISION", "bf16")


def precision() -> str:
    return _precision


def set_precision(p: str) -> None:
    global _precision
    if p not in ("bf16", "fp32"):
        raise ValueError(p)
    _precision = p


@contextlib.contextmanager
def use_precision(p: str):
    old = _precision
    set_precision(p)
    try:
        yield
    finally:
        set_precision(old)


def compute_dtype():
    return torch.bfloat16 if _precision == "bf16" else torch.float32


# --------------------------------------------------------------------------------- weight cache
class _Entry:
    __slots__ = ("version", "tensor", "ptr", "ref")

    def valid_for(self, p) -> bool:
        # id(p) and the allocator's data_ptr are both reused once p is freed: the weak reference is what
        # tells a live parameter from a new one that landed on the same id / address
        return self.ref() is p and self.version == p._version and self.ptr == p.data_ptr()


def _entry(p, tensor) -> _Entry:
    e = _Entry()
    e.version, e.tensor, e.ptr, e.ref = p._version, tensor, p.data_ptr(), weakref.ref(p)
    return e


_wcache: dict = {}
_wcache_gen = 0          # bumped whenever an entry is created, replaced or dropped (optimizer tables check it)
_cache_epoch = 0         # bumped by clear_cache() only: captured HIP graphs key their validity on it
_retained = None         # list collecting every cached tensor handed out while `retaining()` is active


def cache_epoch() -> int:
    return _cache_epoch


@contextlib.contextmanager
def retaining():
    """Collect strong references to every cached weight copy / table served inside the block. A HIP graph captured
    inside reads these buffers by address on every replay, so its owner keeps the list alive (fddm_hip.graphs):
    a later clear_cache() then cannot free memory the graph still reads."""
    global _retained
    old, _retained = _retained, []
    try:
        yield _retained
    finally:
        if old is not None:
            old.extend(_retained)
        _retained = old


def _retain(t):
    if _retained is not None:
        _retained.append(t)
    return t


def wcache_generation() -> int:
    return _wcache_gen


def bf16_entry(p: torch.Tensor):
    """The cached bf16 copy currently served for p (None if there is none)."""
    e = _wcache.get((id(p), torch.bfloat16, None))
    return e.tensor if e is not None and e.ref() is p else None


def wt(p: torch.Tensor, dtype=None, transform=None, key=None) -> torch.Tensor:
    """Return `p` in the compute dtype (cached; refreshed when p changes in place).

    `transform(p) -> tensor` builds a derived layout (e.g. conv weights permuted for the implicit GEMM);
    it is keyed by `key`. fp32 + no transform returns p itself.
    """
    dtype = dtype or compute_dtype()
    if transform is None and dtype == p.dtype and p.is_contiguous():
        return p.detach()
    k = (id(p), dtype, key)
    e = _wcache.get(k)
    if e is not None and e.valid_for(p):
        return _retain(e.tensor)
    with torch.no_grad():
        src = transform(p.detach()) if transform is not None else p.detach()
        src = src.contiguous()
        out = src if src.dtype == dtype else ops.cast(src, dtype)
    global _wcache_gen
    _wcache[k] = _entry(p, out)
    _wcache_gen += 1
    return _retain(out)


def wt_refresh_from(p: torch.Tensor, bf16_copy: torch.Tensor) -> None:
    """Record a bf16 copy written by the fused optimizer as current for `p`."""
    global _wcache_gen
    _wcache[(id(p), torch.bfloat16, None)] = _entry(p, bf16_copy)
    _wcache_gen += 1


def wt_bf16_buffer(p: torch.Tensor) -> torch.Tensor:
    """The cached bf16 copy buffer of p (allocating it), for the optimizer to write in place."""
    k = (id(p), torch.bfloat16, None)
    e = _wcache.get(k)
    if e is None or e.ref() is not p or e.tensor.shape != p.shape:
        return wt(p, torch.bfloat16)
    return e.tensor


def clear_cache():
    global _wcache_gen, _cache_epoch
    _wcache.clear()
    _wcache_gen += 1
    _cache_epoch += 1
    _tables.clear()


# ---------------------------------------------------------------------------------------- seeds
_seed_counter = 0
_base_seed = None


def next_seed() -> int:
    """A fresh dropout seed per forward call (deterministic given torch.initial_seed())."""
    global _base_seed, _seed_counter
    if _base_seed is None:
        _base_seed = int(torch.initial_seed()) & 0xFFFFFFFF
    _seed_counter += 1
    return (_base_seed * 1000003 + _seed_counter) & 0x7FFFFFFFFFFFFFFF


def seed_counter() -> int:
    """The dropout-seed counter (next_seed returns base * 1000003 + counter + 1); graph replays advance it."""
    global _base_seed
    if _base_seed is None:       # fixed now (as next_seed would), not inside a capture
        _base_seed = int(torch.initial_seed()) & 0xFFFFFFFF
    return _seed_counter


def set_seed_counter(c: int) -> None:
    global _seed_counter
    _seed_counter = int(c)


def reseed(seed: int) -> None:
    global _base_seed, _seed_counter
    _base_seed = int(seed) & 0xFFFFFFFF
    _seed_counter = 0


def seed_state() -> list:
    """[base seed, counter] — saved in checkpoints so a resumed run continues the same streams."""
    return [-1 if _base_seed is None else int(_base_seed), int(_seed_counter)]


def set_seed_state(state) -> None:
    global _base_seed, _seed_counter
    b, c = int(state[0]), int(state[1])
    _base_seed = None if b < 0 else b
    _seed_counter = c


# --------------------------------------------------------------------------------------- tables
_tables: dict = {}


def _table_get(k, owner):
    """Cached derived table of `owner` under key k — only while that very tensor is alive (its id is reused
    once it is freed, so the key alone could hand a new model the old one's table)."""
    v = _tables.get(k)
    return _retain(v[1]) if v is not None and v[0]() is owner else None


def _table_put(k, owner, t):
    _tables[k] = (weakref.ref(owner), _retain(t))


def rope_tables(L: int, inv_freq: torch.Tensor, device):
    """cos/sin [L, d] exactly as RoPEEmbedding.forward (models/denoise_decoder.py:35-40), computed on
    the host once per (L, d) and kept resident."""
    k = ("rope", L, id(inv_freq), inv_freq._version, inv_freq.numel(), str(device))  # no device read (graph capture)
    t = _table_get(k, inv_freq)
    if t is None:
        f = inv_freq.detach().float().cpu()
        pos = torch.arange(L, dtype=f.dtype)
        fr = torch.outer(pos, f)
        emb = torch.cat((fr, fr), dim=-1)
        t = (emb.cos().contiguous().to(device), emb.sin().contiguous().to(device))
        _table_put(k, inv_freq, t)
    return t


def rel_bucket(rel: torch.Tensor, num_buckets: int, max_distance: int) -> torch.Tensor:
    """Relative-position buckets, HF modeling_wavlm.py:253-271 (integer-exact host computation)."""
    nb = num_buckets // 2
    buckets = (rel > 0).to(torch.long) * nb
    rel = torch.abs(rel)
    max_exact = nb // 2
    is_small = rel < max_exact
    large = torch.log(rel.float() / max_exact)
    large = large / math.log(max_distance / max_exact)
    large = large * (nb - max_exact)
    large = (max_exact + large).to(torch.long)
    large = torch.min(large, torch.full_like(large, nb - 1))
    return buckets + torch.where(is_small, rel, large)


def relbias_table(S: int, embed: torch.Tensor, num_buckets: int, max_distance: int):
    """[H, 2S-1] fp32: table[h][r] = rel_attn_embed[bucket(r - (S-1))][h]  (r = key - query + S - 1)."""
    k = ("rel", S, id(embed), embed._version, num_buckets, max_distance)
    t = _table_get(k, embed)
    if t is None:
        rel = torch.arange(-(S - 1), S)
        b = rel_bucket(rel, num_buckets, max_distance).to(embed.device)
        t = embed.detach().float()[b].t().contiguous()
        _table_put(k, embed, t)
    return t


# ---------------------------------------------------------------------------------- grad arena
class GradArena:
    """One flat fp32 buffer backing the .grad of parameters that receive a gradient on every step
    (the decoder). Kernels accumulate weight gradients straight into these views (the autograd
    Function returns None for them), one fill zeroes all of them, the fused AdamW walks them in
    place and the DP all-reduce moves the flat buffer without packing. Each slot starts on a 256-B
    boundary. Parameters outside the arena keep torch's None-until-touched semantics (the L_fd
    projectors, whose None grads on non-L_fd steps make AdamW skip them, reference train.py:400-423)."""

    ALIGN = 64

    def __init__(self, params, order=None):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("empty grad arena")
        if order is not None:
            # lay the slots out in the order backward finalises them (head, last block ... first block, rest), so
            # the DP all-reduce can start on a finished prefix while backward still runs (dist.OverlapReducer)
            rank = {id(p): i for i, p in enumerate(order)}
            self.params.sort(key=lambda p: rank.get(id(p), len(rank)))
        offs, n = [], 0
        for p in self.params:
            offs.append(n)
            n += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        dev = self.params[0].device
        self.flat = torch.zeros(n, device=dev, dtype=torch.float32)
        self.offs = offs + [n]
        self.slot = {id(p): i for i, p in enumerate(self.params)}
        self.on_ready = None     # set by dist.OverlapReducer (DP runs): called by grads_ready()
        self.reducer = None
        self.clean = False       # True while the flat buffer is known to be zero (FusedAdamW zero_grads)
        self.views = []
        for p, o in zip(self.params, offs):
            v = self.flat[o:o + p.numel()].view_as(p)
            self.views.append(v)
            p._fddm_arena = self
        self.attach()

    def attach(self):
        """(re)bind every param's .grad to its arena view (after a set_to_none zero_grad)."""
        for p, v in zip(self.params, self.views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def zero_(self):
        self.attach()
        self.flat.zero_()


def grads_ready(params) -> None:
    """Called by a backward Function once the gradients of `params` are final for this step (everything that
    accumulates into their arena slots has been enqueued on the current stream)."""
    for p in params:
        a = getattr(p, "_fddm_arena", None)
        if a is not None and a.on_ready is not None:
            a.on_ready(params)
            return


def grad_slot(p: torch.Tensor):
    """The arena view a kernel should accumulate p's gradient into, or None (autograd returns it)."""
    a = getattr(p, "_fddm_arena", None)
    g = p.grad
    if a is None or g is None or g.dtype != torch.float32:
        return None
    return g


# ------------------------------------------------------------------------------ launch probes
_probes: dict | None = None
_replay_n = 0


@contextlib.contextmanager
def probe(name: str, replay=None):
    """HIP events around one launch site on the current stream, recorded only while
    `probing([...names])` is active (bench.py times its dominant kernel inside the timed steps). With
    `probing(..., replays=n)` and an idempotent `replay` callable (the same launch on the same tensors), the site is
    also launched n more times back to back between a second event pair: the kernel's own duration without the
    launch gap a lone event pair around one short kernel includes (key "<name>#replay", entries (start, end, n))."""
    if _probes is None or name not in _probes:
        yield
        return
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    yield
    e1.record(s)
    _probes[name].append((e0, e1))
    if replay is not None and _replay_n > 0:
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record(s)
        for _ in range(_replay_n):
            replay()
        r1.record(s)
        _probes.setdefault(name + "#replay", []).append((r0, r1, _replay_n))


def probing_any(prefix: str) -> bool:
    """True while probing() collects a launch site whose name starts with `prefix`."""
    return _probes is not None and any(n.startswith(prefix) for n in _probes)


@contextlib.contextmanager
def probing(names, replays=0):
    """Collect probe events for `names`; yields the dict name -> list of (start, end) events."""
    global _probes, _replay_n
    old, old_n = _probes, _replay_n
    _probes = {n: [] for n in names}
    _replay_n = replays
    try:
        yield _probes
    finally:
        _probes, _replay_n = old, old_n
