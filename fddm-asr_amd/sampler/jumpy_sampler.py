"""Jumpy sampling on MI355X (drop-in for sampler/jumpy_sampler.py of the reference).

Same classes, constructor and method signatures as the reference (ModelAdapter, DiffusionJumpySampler:
_mix_with_uniform, _to_indices, _jump_once, _alpha_bar_at_t_train, sample, get_sampling_info).
The denoise step is the decoder forward (libfddm_hip) followed by ONE fused kernel per jump
(csrc/jumpy.hip, `fddm_jump`) that decides x_{t-Δ} from the logits rows in closed form — no one-hot,
softmax or [B, L, K] posterior tensors. `sample(..., graph=True)` captures the whole T_infer/r jump
loop in a HIP graph and replays it.

Reference behaviours kept:
* posterior_mode "max" → argmax; any other mode (incl. the config's "map") → greedy argmax, or a
  Categorical draw when greedy=False (jumpy_sampler.py:212-215, 153-162);
* the decoder sees t in T_infer units (jumpy_sampler.py:187-188) while the exact posterior indexes
  the training schedule's betas at t..t-Δ+1 (diffusion_scheduler.py:146-167, incl. its in-place
  aliasing, see DiscreteDiffusionScheduler.multi_step_coeffs);
* fast mode uses ᾱ at round(t_target / T_infer · T_train) (jumpy_sampler.py:217-233), IndexError at
  T_train included;
* the final decode is argmax of the last x̂0 (jumpy_sampler.py:289-292).
Draws for greedy=False use the build's counter RNG, not torch's Categorical stream.
"""
from __future__ import annotations

from typing import Literal, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from fddm_hip import ops
from fddm_hip import runtime as rt


class ModelAdapter:
    """jumpy_sampler.py:56-88."""

    def __init__(self, decoder):
        self.decoder = decoder

    @torch.no_grad()
    def predict_x0_logits(self, x_t_idx: Tensor, t: Tensor, cond_c: Tensor) -> Tensor:
        return self.decoder(x_t_idx, t, cond_c)


class DiffusionJumpySampler:
    """jumpy_sampler.py:91-307."""

    def __init__(self, scheduler, decoder, K: int, T_train: int, T_infer: int, r: int = 2, greedy: bool = True,
                 posterior_mode: Literal["average", "max"] = "average",
                 sampling_mode: Literal["exact", "fast"] = "exact", temperature: float = 1.0,
                 device: Optional[torch.device] = None):
        self.scheduler = scheduler
        self.model = ModelAdapter(decoder)
        self.K = int(K)
        self.T_train = int(T_train)
        self.T_infer = int(T_infer)
        self.r = int(r)
        self.greedy = bool(greedy)
        self.posterior_mode = posterior_mode
        self.sampling_mode = sampling_mode
        self.temperature = float(temperature)
        self.device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
        alpha_bar = getattr(self.scheduler, "alpha_bar", None)
        if alpha_bar is None:
            raise ValueError("scheduler must provide alpha_bar")
        self.alpha_bar = torch.as_tensor(alpha_bar, dtype=torch.float32, device=self.device)
        self._graphs = {}

    # ----------------------------------------------------------------- reference helpers (torch)
    def _mix_with_uniform(self, p_x0: Tensor, alpha_bar_t: Tensor) -> Tensor:
        B, L, K = p_x0.shape
        u = torch.full((1, 1, K), 1.0 / K, device=p_x0.device, dtype=p_x0.dtype)
        if alpha_bar_t.ndim == 1:
            alpha_bar_t = alpha_bar_t[:, None, None]
        return alpha_bar_t * p_x0 + (1.0 - alpha_bar_t) * u

    def _to_indices(self, probs: Tensor) -> Tensor:
        if self.greedy:
            return probs.argmax(dim=-1)
        if self.temperature != 1.0:
            probs = F.softmax(probs.clamp_min(1e-12).log() / self.temperature, dim=-1)
        return torch.distributions.Categorical(probs=probs).sample()

    def _alpha_bar_at_t_train(self, t_infer_scalar: int) -> Tensor:
        if t_infer_scalar <= 0:
            return torch.tensor(1.0, device=self.device, dtype=torch.float32)
        ratio = float(t_infer_scalar) / float(max(1, self.T_infer))
        t_train_float = max(1.0, min(float(self.T_train), ratio * float(self.T_train)))
        return self.alpha_bar[int(round(t_train_float))]

    # ---------------------------------------------------------------------------- fused step
    def _mode(self) -> int:
        m = ops.JUMP_FAST if self.sampling_mode != "exact" else 0
        if self.posterior_mode != "max" and not self.greedy:
            m |= ops.JUMP_SAMPLE
        return m

    def _coef(self, t_scalar: int, delta: int, B: int) -> Tensor:
        """[B, 4] f32 step coefficients (built before any graph capture)."""
        if self.sampling_mode == "exact":
            tt = torch.full((B,), t_scalar, dtype=torch.long, device=self.scheduler.betas.device)
            delta = min(delta, t_scalar)
            a, b, a_tg, b_tg = self.scheduler.multi_step_coeffs(tt, delta)
            c = torch.stack([a, b, a_tg, b_tg], dim=1).float()
        else:
            ab = self._alpha_bar_at_t_train(max(0, t_scalar - delta)).float()
            c = torch.zeros(B, 4)
            c[:, 0] = float(ab)
        return c.to(self.device).contiguous()

    def _plan(self, B: int):
        plan, t = [], self.T_infer
        while t > 0:
            delta = min(self.r, t)
            plan.append((t, delta, self._coef(t, delta, B)))
            t -= delta
        return plan

    def _step(self, x: Tensor, t_scalar: int, delta: int, cond_c: Tensor, coef: Tensor):
        B, L = x.shape
        t_tensor = torch.full((B,), t_scalar, device=x.device, dtype=torch.long)
        logits = self.model.predict_x0_logits(x, t_tensor, cond_c)
        z = logits.reshape(B * L, -1)
        if z.dtype != torch.float32 or z.stride(-1) != 1:
            z = z.float().contiguous()
        seed = rt.next_seed() if self._mode() & ops.JUMP_SAMPLE else 0
        nx, x0h = ops.jump(z, x.reshape(-1).contiguous(), coef, L, mode=self._mode(), temperature=self.temperature,
                           seed=seed, rng_stream=7)
        return nx.view(B, L), x0h.view(B, L), logits

    def _run(self, x: Tensor, cond_c: Tensor, plan):
        x0h = logits = None
        for t, delta, coef in plan:
            x, x0h, logits = self._step(x, t, delta, cond_c, coef)
        return x, x0h, logits

    @torch.no_grad()
    def _jump_once(self, x_t_idx: Tensor, t_scalar: int, delta: int, cond_c: Tensor,
                   seq_len: int) -> Tuple[Tensor, Tensor]:
        """jumpy_sampler.py:167-215: returns (x_{t-Δ} [B, L], p_x0 [B, L, K])."""
        coef = self._coef(t_scalar, delta, x_t_idx.shape[0])
        nx, _, logits = self._step(x_t_idx, t_scalar, delta, cond_c, coef)
        return nx, F.softmax(logits.float(), dim=-1)

    # -------------------------------------------------------------------------- public API
    @torch.no_grad()
    def sample(self, cond_c: Tensor, seq_len: int, init: Literal["uniform", "random"] = "uniform",
               graph: bool = False, return_probs: bool = True) -> Tuple[Tensor, Optional[Tensor]]:
        """jumpy_sampler.py:238-293: x_T ~ U{0..K-1}, jump by Δ = min(r, t) until t = 0; returns
        (argmax x̂0 of the last jump [B, L], p_x0_last [B, L, K] or None when return_probs=False).
        graph=True replays the whole loop from a captured HIP graph (captured on first use per shape)."""
        B = cond_c.size(0)
        device = cond_c.device
        x_T = torch.randint(low=0, high=self.K, size=(B, seq_len), device=device)
        if graph:
            x0, logits = self._sample_graph(x_T, cond_c)
        else:
            _, x0, logits = self._run(x_T, cond_c, self._plan(B))
        if not return_probs:
            return x0, None
        return x0, F.softmax(logits.float(), dim=-1)

    def _sample_graph(self, x_T: Tensor, cond_c: Tensor):
        B, L = x_T.shape
        key = (B, L, tuple(cond_c.shape[1:]), cond_c.dtype, self.T_infer, self.r, self._mode(), self.temperature)
        ent = self._graphs.get(key)
        if ent is None:
            plan = self._plan(B)
            sx, sc = x_T.clone(), cond_c.detach().clone()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):       # warm-up: weight caches, RoPE tables, library handles
                self._run(sx, sc, plan)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                _, x0, logits = self._run(sx, sc, plan)
            ent = (g, sx, sc, x0, logits)
            self._graphs[key] = ent
        g, sx, sc, x0, logits = ent
        sx.copy_(x_T)
        sc.copy_(cond_c)
        g.replay()
        return x0.clone(), logits

    def get_sampling_info(self) -> dict:
        return {"sampling_mode": self.sampling_mode, "posterior_mode": self.posterior_mode, "T_infer": self.T_infer,
                "r": self.r, "greedy": self.greedy, "temperature": self.temperature, "K": self.K}
