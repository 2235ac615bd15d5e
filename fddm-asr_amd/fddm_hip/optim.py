"""Fused clip_grad_norm_ + AdamW (train.py:411-423) over libfddm_hip: two launches per step, no
host synchronisation, and the bf16 weight copies for the next forward written in the same pass."""
from __future__ import annotations

import math

import torch

from . import runtime as rt
from ._lib import call
from .ops import stream

CHUNK = 65536


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW semantics (decoupled weight decay, bias-corrected moments, per-parameter step
    counts; parameters whose .grad is None are skipped entirely, as with set_to_none=True)."""

    def __init__(self, params, lr=2e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._tables = {}
        self._ring = None        # pinned host slots for the per-step bias-correction scalars (see _upload)
        self._ring_i = 0
        self.last_total_sq = None
        self.arena = None

    def use_grad_arena(self, params, order=None):
        """Back the grads of `params` (parameters that get a gradient every step) by one flat buffer
        (runtime.GradArena, slots laid out in `order` if given); zero_grad() then zeroes it with a single fill
        instead of dropping grads."""
        self.arena = rt.GradArena(params, order)
        return self.arena

    def zero_grad(self, set_to_none: bool = True):
        if self.arena is None:
            return super().zero_grad(set_to_none)
        inside = set(id(p) for p in self.arena.params)
        for group in self.param_groups:
            for p in group["params"]:
                if id(p) not in inside and p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()
        self.arena.zero_()

    def _table(self, group, plist):
        dev = plist[0].device
        cd = rt.compute_dtype()
        key = (id(group),) + tuple((p.data_ptr(), p.grad.data_ptr()) for p in plist) + (cd,)
        t = self._tables.get(key)
        if t is not None:
            return t
        if len(self._tables) >= 8:  # the train step alternates between a few parameter sets (L_fd steps add the
            self._tables.clear()    # projectors): keep each set's device table instead of rebuilding it per switch
        ct, cs, numel, pp, gp, mp, vp, bp = [], [], [], [], [], [], [], []
        for i, p in enumerate(plist):
            st = self.state[p]
            n = p.numel()
            for s0 in range(0, n, CHUNK):
                ct.append(i)
                cs.append(s0)
            numel.append(n)
            pp.append(p.data_ptr())
            gp.append(p.grad.data_ptr())
            mp.append(st["exp_avg"].data_ptr())
            vp.append(st["exp_avg_sq"].data_ptr())
            if cd == torch.bfloat16 and p.dim() >= 2:
                bp.append(rt.wt_bf16_buffer(p).data_ptr())
            else:
                bp.append(0)
        L = lambda v: torch.tensor(v, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)  # noqa: E731
        tab = dict(ct=L(ct), cs=L(cs), numel=L(numel), p=L(pp), g=L(gp), m=L(mp), v=L(vp), b=L(bp), n=len(ct))
        self._tables[key] = tab
        return tab

    def _upload(self, vals, dev):
        """Host floats -> device f32 tensor through a ring of reused pinned slots (no pinned allocation per step);
        a slot is reused only after the copy that last read it has completed (its event)."""
        R, n = 8, len(vals)
        if self._ring is None or self._ring[0].shape[1] < n:
            cap = max(n, 256)
            self._ring = (torch.empty(R, cap, dtype=torch.float32).pin_memory(), [None] * R,
                          torch.empty(R, cap, dtype=torch.float32, device=dev))
        host, evs, devbuf = self._ring
        i = self._ring_i % R
        self._ring_i += 1
        if evs[i] is not None:
            evs[i].synchronize()
        host[i, :n] = torch.tensor(vals, dtype=torch.float32)
        out = devbuf[i, :n]
        out.copy_(host[i, :n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        evs[i] = ev
        return out

    @torch.no_grad()
    def clip_and_step(self, max_norm: float | None = None):
        """clip_grad_norm_(all params with grads, max_norm) followed by AdamW.step(); returns the
        (device) total gradient norm."""
        groups = []
        for group in self.param_groups:
            plist = [p for p in group["params"] if p.grad is not None]
            if not plist:
                continue
            for p in plist:
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    p.grad = p.grad.float().contiguous()
            groups.append((group, plist, self._table(group, plist)))
        if not groups:
            return None
        dev = groups[0][1][0].device
        total = None
        if max_norm is not None:
            total = torch.zeros(1, device=dev, dtype=torch.float32)
            for group, plist, tab in groups:
                call("fddm_grad_sumsq", tab["ct"].data_ptr(), tab["cs"].data_ptr(), tab["numel"].data_ptr(),
                     tab["g"].data_ptr(), tab["n"], total.data_ptr(), stream())
        for group, plist, tab in groups:
            b1, b2 = group["betas"]
            ss, b2s = [], []
            for p in plist:
                st = self.state[p]
                st["step"] += 1
                ss.append(group["lr"] / (1 - b1 ** st["step"]))
                b2s.append(math.sqrt(1 - b2 ** st["step"]))
            sb = self._upload(ss + b2s, dev)      # one copy for both per-tensor scalar arrays
            ss_t, b2_t = sb[: len(ss)], sb[len(ss):]
            call("fddm_adamw", tab["ct"].data_ptr(), tab["cs"].data_ptr(), tab["numel"].data_ptr(), tab["p"].data_ptr(),
                 tab["g"].data_ptr(), tab["m"].data_ptr(), tab["v"].data_ptr(), tab["b"].data_ptr(), ss_t.data_ptr(),
                 b2_t.data_ptr(), tab["n"], total.data_ptr() if total is not None else 0,
                 float(max_norm or 0.0), float(group["lr"] * group["weight_decay"]), float(b1), float(b2),
                 float(group["eps"]), stream())
        self.last_total_sq = total
        return None if total is None else total.sqrt()

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.clip_and_step(None)
        return loss
