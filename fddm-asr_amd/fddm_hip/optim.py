"""Fused clip_grad_norm_ + AdamW (train.py:411-423) over libfddm_hip: three launches per step, no
host synchronisation, and the bf16 weight copies for the next forward written in the same pass.

`state["step"]` is a 0-d fp32 tensor on the parameter's device (torch.optim.AdamW keeps a 0-d fp32 tensor
too; its capturable/fused variants keep it on the device), advanced by the kernel, so a step skipped by the
non-finite guard (GradScaler semantics, reference train.py:401-413) leaves the bias corrections exact."""
from __future__ import annotations

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
        self.table_epoch = 0     # bumped whenever a chunk table is (re)built: captured step graphs key on it
        self.last_total_sq = None
        self.arena = None
        self.aux_arena = None
        self._skipped = None     # device int32: steps skipped by the non-finite guard

    def use_grad_arena(self, params, order=None):
        """Back the grads of `params` (parameters that get a gradient every step) by one flat buffer
        (runtime.GradArena, slots laid out in `order` if given); zero_grad() then zeroes it with a single fill
        instead of dropping grads."""
        self.arena = rt.GradArena(params, order)
        return self.arena

    def use_aux_arena(self, params):
        """Back the grads of `params` that get a gradient only on some steps (the L_fd projectors, train.py:372-397)
        by a second flat buffer: zero_grad() still leaves them None (AdamW skips them on KL-only steps, the reference's
        set_to_none semantics) and attach_aux() binds them to their zeroed views on the steps that produce them, so
        their gradient buffers keep one address (the kernels accumulate into them; the optimizer's chunk table and a
        captured step graph stay valid). The fused AdamW's zero_grads pass leaves the views zeroed again."""
        self.aux_arena = rt.GradArena(params)
        self.aux_arena.views_zero = True
        for p in self.aux_arena.params:
            p.grad = None
        return self.aux_arena

    def attach_aux(self):
        a = self.aux_arena
        if a is None:
            return
        if not getattr(a, "views_zero", False):
            a.flat.zero_()
        a.attach()
        a.views_zero = False

    def zero_grad(self, set_to_none: bool = True):
        if self.arena is None:
            return super().zero_grad(set_to_none)
        clean = self.arena.clean
        self.arena.clean = False
        inside = set(id(p) for p in self.arena.params)
        for group in self.param_groups:
            for p in group["params"]:
                if id(p) not in inside and p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()
        if clean:           # the last clip_and_step(zero_grads=True) left the arena zeroed in its own pass
            self.arena.attach()
        else:
            self.arena.zero_()
        if self.aux_arena is not None and set_to_none:
            for p in self.aux_arena.params:
                p.grad = None

    @staticmethod
    def _bufs_live(plist, bufs) -> bool:
        """The bf16 copies a table writes are still the runtime cache's live entries for their parameters."""
        for p, b in zip(plist, bufs):
            if b is not None and rt.bf16_entry(p) is not b:
                return False
        return True

    def _table(self, group, plist):
        dev = plist[0].device
        cd = rt.compute_dtype()
        key = (id(group),) + tuple((p.data_ptr(), p.grad.data_ptr(), self.state[p]["step"].data_ptr())
                                   for p in plist) + (cd,)
        t = self._tables.get(key)
        if t is not None:
            # the runtime replaced or dropped cached bf16 copies since the table was built (clear_cache, a
            # parameter changed in place): rebuild, so the kernel never writes a copy the forward no longer reads
            if t["gen"] == rt.wcache_generation():
                return t
            if self._bufs_live(plist, t["bufs"]):
                t["gen"] = rt.wcache_generation()
                return t
            del self._tables[key]
            self.table_epoch += 1   # a table a captured step may read was replaced
        if len(self._tables) >= 8:  # the train step alternates between a few parameter sets (L_fd steps add the
            self._tables.clear()    # projectors): keep each set's device table instead of rebuilding it per switch
            self.table_epoch += 1
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("FusedAdamW: a chunk table would be built inside a HIP-graph capture (its host-to-"
                               "device copy cannot be captured); run one eager step of this parameter set first")
        ct, cs, numel, pp, gp, mp, vp, bp, sp, bufs = [], [], [], [], [], [], [], [], [], []
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
            sp.append(st["step"].data_ptr())
            if cd == torch.bfloat16 and p.dim() >= 2:
                b = rt.wt_bf16_buffer(p)
                bufs.append(b)               # held by the table: the kernel never writes freed memory
                bp.append(b.data_ptr())
            else:
                bufs.append(None)
                bp.append(0)
        L = lambda v: torch.tensor(v, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)  # noqa: E731
        tab = dict(ct=L(ct), cs=L(cs), numel=L(numel), p=L(pp), g=L(gp), m=L(mp), v=L(vp), b=L(bp), s=L(sp),
                   n=len(ct), nt=len(plist), bufs=bufs, gen=rt.wcache_generation())
        self._tables[key] = tab
        return tab

    def _init_state(self, p):
        st = self.state[p]
        if not st:
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        elif not (torch.is_tensor(st["step"]) and st["step"].device == p.device and st["step"].dtype == torch.float32
                  and st["step"].dim() == 0):
            st["step"] = torch.tensor(float(st["step"]), dtype=torch.float32, device=p.device)
        return st

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._tables.clear()
        self.table_epoch += 1
        for group in self.param_groups:
            for p in group["params"]:
                if self.state.get(p):
                    self._init_state(p)

    def skipped_steps(self):
        """Device int32 count of steps skipped by the non-finite guard (None before the first step)."""
        return self._skipped

    @torch.no_grad()
    def clip_and_step(self, max_norm: float | None = None, zero_grads: bool = False, grad_scale: float = 1.0,
                      return_norm: bool = True):
        """clip_grad_norm_(all params with grads, max_norm) followed by AdamW.step(); returns the
        (device) total gradient norm (return_norm=False: None, and no sqrt launch — the sum of squares stays in
        last_total_sq). zero_grads: the step also zeroes every gradient it reads (the train loop's
        next zero_grad then has no arena fill to do; .grad reads as zero after the call). grad_scale: every gradient
        is multiplied by it before the clip and the update (data parallelism: the all-reduce leaves the ranks' sum,
        grad_scale = 1/W averages it inside the kernel instead of a pass over the gradients)."""
        groups = []
        for group in self.param_groups:
            plist = [p for p in group["params"] if p.grad is not None]
            if not plist:
                continue
            for p in plist:
                self._init_state(p)
                if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    p.grad = p.grad.float().contiguous()
            groups.append((group, plist, self._table(group, plist)))
        if not groups:
            return None
        dev = groups[0][1][0].device
        if self._skipped is None:
            self._skipped = torch.zeros(1, device=dev, dtype=torch.int32)
        # the gradient sum of squares feeds both the clip coefficient and the non-finite guard
        total = torch.zeros(1, device=dev, dtype=torch.float32)
        for group, plist, tab in groups:
            call("fddm_grad_sumsq", tab["ct"].data_ptr(), tab["cs"].data_ptr(), tab["numel"].data_ptr(),
                 tab["g"].data_ptr(), tab["n"], total.data_ptr(), stream())
        for gi, (group, plist, tab) in enumerate(groups):
            b1, b2 = group["betas"]
            call("fddm_adamw", tab["ct"].data_ptr(), tab["cs"].data_ptr(), tab["numel"].data_ptr(), tab["p"].data_ptr(),
                 tab["g"].data_ptr(), tab["m"].data_ptr(), tab["v"].data_ptr(), tab["b"].data_ptr(), tab["s"].data_ptr(),
                 tab["nt"], tab["n"], total.data_ptr(), float(max_norm or 0.0), float(group["lr"]),
                 float(group["lr"] * group["weight_decay"]), float(b1), float(b2), float(group["eps"]),
                 self._skipped.data_ptr() if gi == 0 else 0, int(bool(zero_grads)), float(grad_scale),
                 stream())   # skip counted once
        if zero_grads and self.arena is not None:
            # every arena slot was in a table AND each .grad is still the arena view the kernel just zeroed (a grad
            # rebound above or by user code leaves its arena slot holding this step's values: zero_grad must fill)
            a = self.arena
            self.arena.clean = all(p.grad is not None and p.grad.data_ptr() == v.data_ptr()
                                   for p, v in zip(a.params, a.views))
        if self.aux_arena is not None:
            a = self.aux_arena
            used = [p.grad is not None for p in a.params]
            if any(used):   # zeroed by this pass only when every view was read through its own address
                a.views_zero = bool(zero_grads) and all(
                    p.grad is not None and p.grad.data_ptr() == v.data_ptr() for p, v in zip(a.params, a.views))
        self.last_total_sq = total
        if not return_norm:
            return None
        return total.sqrt() * grad_scale if grad_scale != 1.0 else total.sqrt()

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.clip_and_step(None)
        return loss
