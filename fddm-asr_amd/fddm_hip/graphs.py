"""HIP-graph replay of the frozen encoder's forward (the host side of the train step was the bottleneck: ~110
launches per batch for the encoder alone, each paying Python + ctypes + HIP launch cost on the host).

The WavLM forward is static for a given (batch shape, precision, persistent-GEMM cap): no randomness, no autograd, no
host synchronisation. It is captured once per shape into two graphs around the conv-layer-1 launch —
stage_conv0 (GroupNorm statistics + conv0 + GELU) and stage_rest (conv layers 2..6, feature projection,
positional conv, 12 transformer layers, encoder.proj) — with conv layer 1 launched eagerly between them, so the
benchmark's HIP-event probe of that dominant launch (runtime.probe) stays an ordinary timed launch. Replaying a
batch is then 1 copy + 2 graph launches + 1 kernel launch instead of ~110 launches.

Slots: the train loop encodes batch i+1 on a side stream while step i's decoder reads batch i's condition, so the
static output buffers alternate between two slots, each with its own input / intermediate / output buffers, graphs
and private memory pool. The pool is NOT shared across slots: a graph captured later may place its output in memory
an earlier capture used for intermediates, so with one pool, replaying slot 0 for batch i+2 would overwrite slot 1's
output while step i+1 still reads it (tools/graph_check2.py reproduces that). Within a slot, gC may reuse gA's
intermediates: the two always replay in capture order and gA's live output (h0) is never reused.
"""
from __future__ import annotations

import weakref
from types import SimpleNamespace

import torch

from . import runtime as rt


class GraphedEncoder:
    def __init__(self, encoder, nslots: int = 2):
        self._enc = weakref.ref(encoder)       # the train loop keeps these per encoder in a WeakKeyDictionary
        self.nslots = nslots
        self.cache: dict = {}

    @staticmethod
    def supported(encoder) -> bool:
        return getattr(encoder, "pooling", "none") == "none" and hasattr(encoder, "backbone") and \
            hasattr(encoder.backbone, "stage_rest")

    @property
    def enc(self):
        return self._enc()

    def _capture(self, wave):
        bb = self.enc.backbone
        inp = wave.detach().clone()
        # eager warm-up: every cached table / prepared weight exists before capture (no host copies inside)
        h0 = bb.stage_conv0(inp)
        h1 = bb.stage_conv1(h0)
        self.enc.project(bb.stage_rest(h1))
        # the runtime-cached tensors the captured launches read (the relative-bias table, the bf16 encoder.proj
        # weight, ...) are held by the slot, so rt.clear_cache() cannot free memory a replay reads
        with rt.retaining() as keep:
            gA = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gA):
                h0 = bb.stage_conv0(inp)
            h1 = torch.empty(bb.conv_out_shape(h0), device=h0.device, dtype=h0.dtype)
            gC = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gC, pool=gA.pool()):      # this slot's pool only (see the module docstring)
                out = self.enc.project(bb.stage_rest(h1))
        return SimpleNamespace(inp=inp, h0=h0, h1=h1, out=out, gA=gA, gC=gC, keep=keep)

    def _weights_token(self):
        """Identity of the weights the graphs read: the backbone's prepared (cast / permuted) weight set — rebuilt
        when the module is moved, loaded or changed in place — encoder.proj, and the runtime cache epoch. A change
        drops every captured graph (they would read freed or stale buffers) and the next run recaptures."""
        enc = self.enc
        P = enc.backbone._prepared(rt.compute_dtype())
        proj = getattr(enc, "proj", None)
        pw = getattr(proj, "weight", None) if getattr(enc, "use_proj", False) else None
        # rt.cache_epoch(): a clear_cache() (load_checkpoint calls it) drops every capture, so the next run recaptures
        # against freshly built tables instead of replaying stale ones
        return (id(P), None if pw is None else (pw.data_ptr(), pw._version), rt.cache_epoch()), P

    @torch.no_grad()
    def run(self, wave, slot: int, cap: int = 0):
        """The encoder's features for `wave` in slot `slot`'s static output buffer (valid until this slot is run
        again), on the current stream."""
        tok, P = self._weights_token()
        if tok != getattr(self, "_tok", None):
            self.cache.clear()
            self._tok, self._P = tok, P          # the captured launches read these buffers: keep them alive
        key = (tuple(wave.shape), wave.dtype, str(wave.device), rt.precision(), int(cap),
               int(getattr(self.enc.backbone, "conv_cus", 0)),
               int(getattr(self.enc.backbone, "conv_cus_rest", 0)))   # grid sizes are part of the captured launches
        slots = self.cache.setdefault(key, [None] * self.nslots)
        s = slots[slot]
        if s is None:
            s = slots[slot] = self._capture(wave)
        s.inp.copy_(wave, non_blocking=True)
        s.gA.replay()
        self.enc.backbone.stage_conv1(s.h0, out=s.h1)
        s.gC.replay()
        return s.out


class StepGraphs:
    """HIP-graph replay of the decoder's train step (reference train.py:340-443 from the decoder forward to the
    optimizer step): decoder forward, KL, the L_fd branch, backward, clip + AdamW — ~230 (C2) / ~450 (C4) launches
    per step enqueued from Python — captured once per step kind (KL-only / L_fd) and replayed as one graph launch.

    The train loop runs the FIRST step of each kind eagerly (its launches create every cached weight copy, table,
    optimizer chunk table and gradient-arena binding the step reads), then captures that kind right away (capture
    executes nothing); later steps of the kind copy their inputs (condition c, x0, t, x_t) into the graphs' static
    buffers and replay. Inputs stay eager: q_sample and the t draw run before the replay, so user schedulers and
    t-draws keep working.

    Dropout seeds: the captured launches read their seed as seed + *off (fddm_set_seed_offset, common.h eff_seed).
    At capture the seed counter is restored afterwards (capturing draws no seeds); before a replay `off` is filled
    with (counter now - counter at capture) and the counter is advanced by the number of seeds the step draws, so a
    replayed step uses exactly the seeds — and dropout masks — an eager step would.

    Validity: a graph reads parameters, cached bf16 weights, optimizer moments / chunk tables and gradient-arena views
    by address. It is dropped (and the step runs eagerly, then recaptures) when the runtime cache epoch changes
    (clear_cache), when any trainable parameter is replaced or changed by a torch op (data_ptr / _version), when
    the optimizer rebuilt its tables (FusedAdamW.table_epoch), when an optimizer hyperparameter the AdamW launch
    takes by value changed (lr, weight decay, betas, eps: `_hparams`) or when the clip_and_step arguments the step
    passes changed (max_norm, grad_scale: the caller's `step_args`). The two kinds share one memory pool (they
    replay on one stream, never concurrently; their outputs stay live).

    Fixed shapes only: the graphs are keyed by the step's input shapes, and a batch of another shape drops both kinds
    (reset) and runs eagerly. With variable-length batches (the real-data loader's per-batch padding) nearly every
    step would capture again and none would replay; bucket the batches to a few fixed shapes before enabling it."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.graphs: dict = {}
        self.static: dict = {}
        self.pool = None
        self.off = torch.zeros(1, device=self.device, dtype=torch.int64)

    def reset(self):
        """Drop every graph; their memory pool goes with them (a new capture starts a new pool)."""
        self.graphs.clear()
        self.static.clear()
        self.pool = None

    @staticmethod
    def _hparams(optimizer):
        """The optimizer hyperparameters a captured AdamW launch bakes in as kernel arguments (lr, weight decay,
        betas, eps per param group): a change (e.g. an lr schedule writing param_groups[i]['lr']) must recapture, or
        replays would keep the captured values. max_norm / grad_scale are clip_and_step() arguments, not optimizer
        state: the caller passes the values its step uses as `step_args`, and they join the token too."""
        return tuple((float(g.get("lr", 0.0)), float(g.get("weight_decay", 0.0)),
                      tuple(float(b) for b in g.get("betas", ())), float(g.get("eps", 0.0)))
                     for g in getattr(optimizer, "param_groups", ()))

    def _token(self, params, optimizer, step_args):
        return (rt.cache_epoch(), getattr(optimizer, "table_epoch", 0), self._hparams(optimizer), tuple(step_args),
                tuple((p.data_ptr(), p._version) for p in params))

    def get(self, kind, params, optimizer, shapes, step_args=()):
        s = self.graphs.get(kind)
        if s is None:
            return None
        if s.shapes != shapes or s.token != self._token(params, optimizer, step_args):
            self.reset()             # stale addresses: recapture both kinds
            return None
        return s

    def capture(self, kind, fn, inputs: dict, params, optimizer, step_args=()):
        """Capture fn(**static inputs) -> tuple of output tensors as step kind `kind`; step_args: the by-value
        arguments fn passes to the optimizer step (clip_and_step's max_norm, grad_scale)."""
        from ._lib import lib
        shapes = tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(inputs.items()))
        if any(self.static.get(k) is None or self.static[k].shape != v.shape or self.static[k].dtype != v.dtype
               for k, v in inputs.items()):
            self.reset()
            self.static = {k: torch.empty_like(v) for k, v in inputs.items()}
        for k, v in inputs.items():
            self.static[k].copy_(v)
        c0 = rt.seed_counter()
        g = torch.cuda.CUDAGraph()
        with rt.retaining() as keep:
            lib().fddm_set_seed_offset(self.off.data_ptr())
            try:
                with torch.cuda.graph(g, pool=self.pool):
                    outs = fn(**self.static)
            finally:
                lib().fddm_set_seed_offset(None)
        nseeds = rt.seed_counter() - c0
        rt.set_seed_counter(c0)
        if self.pool is None:
            self.pool = g.pool()
        self.graphs[kind] = SimpleNamespace(g=g, outs=outs, c0=c0, nseeds=nseeds, keep=keep, shapes=shapes,
                                            token=self._token(params, optimizer, step_args))

    def replay(self, kind, inputs: dict):
        s = self.graphs[kind]
        for k, v in inputs.items():
            self.static[k].copy_(v, non_blocking=True)
        c = rt.seed_counter()
        self.off.fill_(c - s.c0)
        rt.set_seed_counter(c + s.nseeds)
        s.g.replay()
        return s.outs
