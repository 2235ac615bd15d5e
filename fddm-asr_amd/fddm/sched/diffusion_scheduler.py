"""DiscreteDiffusionScheduler (drop-in for fddm/sched/diffusion_scheduler.py of the reference).

Same constructor, attributes (K, T, device, eps, betas, alpha_bar, w_prefix) and methods. The
train-step path uses two fused MI355X entry points that SchedulerAdapter dispatches to:
  * sample_xt(x0, t, seed): q_sample + torch.multinomial in one kernel — a closed-form inverse CDF
    over the two distinct q(x_t|x_0) probabilities (bit-exact with the CPU oracle's RNG contract);
  * the categorical KL is in fddm_hip.functions.KLFn.
q_sample / q_posterior / q_posterior_multi_step are kept (device-generic torch) for the sampler and
evaluation callers; their math follows diffusion_scheduler.py:31-208 (the multi-step coefficients
are computed with a vectorised recurrence instead of per-element .item() loops).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from fddm_hip import ops


class DiscreteDiffusionScheduler:
    def __init__(self, K: int, T: int, device: torch.device, beta_max: float = 0.2, eps: float = 1e-8):
        self.K = int(K)
        self.T = int(T)
        self.device = device
        self.eps = float(eps)
        t = torch.arange(1, T + 1, device=device, dtype=torch.float32)
        self.betas = beta_max * torch.sin(0.5 * math.pi * (t / float(T))) ** 2           # :26
        self.alpha_bar = torch.cumprod(1.0 - self.betas, dim=0)                         # :28
        self._thr = None

    # ---------------------------------------------------------------- fused train-step sampler
    def sample_thresholds(self) -> torch.Tensor:
        """uint32 P(x_t = x_0) thresholds per t: floor(p_hi * 2^32), p_hi from q_sample's clamp +
        renormalisation (diffusion_scheduler.py:45-49) in fp32."""
        if self._thr is None:
            ab = self.alpha_bar.detach().float().cpu()
            u = torch.tensor(1.0 / self.K, dtype=torch.float32)
            hi = (ab + (1.0 - ab) * u).clamp_min(self.eps)
            lo = ((1.0 - ab) * u).clamp_min(self.eps)
            s = (hi.double() + (self.K - 1) * lo.double()).float().clamp_min(self.eps)
            p = (hi / s).double().numpy()
            thr = np.clip(np.floor(p * 4294967296.0), 0, 4294967295).astype(np.uint32)
            self._thr = torch.from_numpy(thr.view(np.int32)).to(self.betas.device)
        return self._thr

    def sample_xt(self, x0: torch.Tensor, t: torch.Tensor, seed: int) -> torch.Tensor:
        return ops.sample_q(x0.contiguous(), t.contiguous().long(), self.sample_thresholds(), self.K, seed)

    # ---------------------------------------------------------------- reference API (torch)
    @torch.no_grad()
    def q_sample(self, x0_prob: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        x0_prob = x0_prob.to(self.device).float()
        t = t.to(self.device).long()
        B, L, K = x0_prob.shape
        assert K == self.K
        ab = self.alpha_bar[t - 1].view(B, 1, 1)
        xt = ab * x0_prob + (1.0 - ab) * torch.full_like(x0_prob, 1.0 / self.K)
        xt = xt.clamp_min(self.eps)
        return xt / xt.sum(dim=-1, keepdim=True).clamp_min(self.eps)

    def _beta_prev(self, t):
        return torch.where((t - 1) == 0, torch.zeros_like(self.betas[t - 1]), self.betas[(t - 2).clamp(min=0)])

    @torch.no_grad()
    def q_posterior(self, xt_prob: torch.Tensor, x0hat_prob: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        xt_prob = xt_prob.to(self.device).float()
        x0hat_prob = x0hat_prob.to(self.device).float()
        t = t.to(self.device).long()
        B, L, K = xt_prob.shape
        assert K == self.K
        bt = self.betas[t - 1].view(B, 1, 1)
        bp = self._beta_prev(t).view(B, 1, 1)
        A = (1.0 - bt) * xt_prob + bt / self.K
        Bv = (1.0 - bp) * x0hat_prob + bp / self.K
        denom = (1.0 - bt) * (xt_prob * x0hat_prob).sum(-1, keepdim=True) + bt / self.K
        post = (A * Bv) / denom.clamp_min(self.eps)
        return post / post.sum(-1, keepdim=True).clamp_min(self.eps)

    def multi_step_coeffs(self, t: torch.Tensor, delta: int):
        """(a_cum, b_cum) of M_{t:t-delta+1} and (a_tgt, b_tgt) of M_{t-delta}, fp32 recurrence over
        s = t .. t-delta+1 as the reference executes it (diffusion_scheduler.py:146-167):
        a' = a_s a, b' = a_s b + b_s (a' + K b). Note a' (not a) in the b update: the reference reads
        `a_old` as a 0-d view of a_cumulative, which the preceding in-place store has already updated."""
        B = t.shape[0]
        a = torch.ones(B, device=self.device)
        b = torch.zeros(B, device=self.device)
        for i in range(delta):
            s = t - i
            valid = (s >= 1) & (s <= self.T)
            bs = self.betas[(s - 1).clamp(0, self.T - 1)]
            a_s, b_s = 1.0 - bs, bs / self.K
            na = a_s * a
            nb = a_s * b + b_s * (na + self.K * b)
            a, b = torch.where(valid, na, a), torch.where(valid, nb, b)
        tt = (t - delta).clamp(min=0)
        btg = self.betas[(tt - 1).clamp(0, self.T - 1)]
        a_tg = torch.where(tt > 0, 1.0 - btg, torch.ones_like(btg))
        b_tg = torch.where(tt > 0, btg / self.K, torch.zeros_like(btg))
        return a, b, a_tg, b_tg

    @torch.no_grad()
    def q_posterior_multi_step(self, xt_prob, x0hat_prob, t, delta: int):
        xt_prob = xt_prob.to(self.device).float()
        x0hat_prob = x0hat_prob.to(self.device).float()
        t = t.to(self.device).long()
        B, L, K = xt_prob.shape
        assert K == self.K
        delta = min(delta, int(t.min().item()))
        if delta <= 0:
            return xt_prob
        a, b, a_tg, b_tg = (v.view(B, 1, 1) for v in self.multi_step_coeffs(t, delta))
        sxt = xt_prob.sum(-1, keepdim=True)
        sx0 = x0hat_prob.sum(-1, keepdim=True)
        A = a * xt_prob + b * sxt
        Bt = a_tg * x0hat_prob + b_tg * sx0
        denom = a * (xt_prob * x0hat_prob).sum(-1, keepdim=True) + b * sx0 * sxt
        post = (A * Bt) / denom.clamp_min(self.eps)
        return post / post.sum(-1, keepdim=True).clamp_min(self.eps)

    @property
    def w_prefix(self):
        return self.alpha_bar
