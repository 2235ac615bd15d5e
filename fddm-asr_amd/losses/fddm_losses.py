"""L_fd cross-modal feature decorrelation (drop-in for losses/fddm_losses.py, lines 18-58).

lfd_loss keeps the reference signature and assertion; the standardisation, the [D x D]
cross-correlation (MFMA GEMM over B*T rows) and the loss/gradient run on libfddm_hip.

Additive keyword `group` (a torch.distributed process group): under data parallelism the batch-dim
statistics span every rank's rows, so an N-rank step computes the loss of the global batch exactly as one
process would (functions.LfdFn). Default None: the batch the caller holds (the reference's
single-process semantics; under DP that is the documented "local-batch L_fd").
"""
from __future__ import annotations

from typing import Tuple

import torch

from fddm_hip import functions as FN


def _standardize(x: torch.Tensor, eps: float = 1e-5) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Reference helper (fddm_losses.py:18-27), kept for API compatibility (torch ops)."""
    mean = x.mean(dim=0, keepdim=True)
    var = x.var(dim=0, unbiased=False, keepdim=True)
    std = torch.sqrt(var + eps)
    return (x - mean) / std, mean, std


def lfd_loss(z_a: torch.Tensor, z_b: torch.Tensor, lambda_offdiag: float = 5.0e-3, eps: float = 1e-5, *,
             group=None) -> torch.Tensor:
    B, T, D = z_a.shape
    assert z_b.shape == (B, T, D), "z_b must have the same shape as z_a"
    return FN.LfdFn.apply(z_a, z_b, float(lambda_offdiag), float(eps), group)
