"""L_fd projection heads (drop-in for models/projection.py of the reference, lines 14-55).

Same classes, constructor arguments and state_dict keys (`proj.net.0.*`, `proj.weight`); the
Linear layers and the softmax·W TextEmbedding run on libfddm_hip (fddm_hip.functions).
"""
from __future__ import annotations

from typing import Literal

import torch
import torch.nn as nn

from fddm_hip import functions as FN


class MLP(nn.Module):
    def __init__(self, dim_in: int, dim_out: int, hidden: int = 0, act: Literal["gelu", "relu"] = "gelu"):
        super().__init__()
        if hidden > 0:
            layers = [nn.Linear(dim_in, hidden), nn.GELU() if act == "gelu" else nn.ReLU(), nn.Linear(hidden, dim_out)]
        else:
            layers = [nn.Linear(dim_in, dim_out)]
        self.net = nn.Sequential(*layers)

    def forward(self, x):
        for m in self.net:
            if isinstance(m, nn.Linear):
                x = FN.linear(x, m.weight, m.bias)
            else:
                x = m(x)
        return x


class SpeechProjector(nn.Module):
    def __init__(self, d_in: int, d_proj: int, hidden: int = 0):
        super().__init__()
        self.proj = MLP(d_in, d_proj, hidden)

    def forward(self, c: torch.Tensor) -> torch.Tensor:
        return self.proj(c)


class TextEmbedding(nn.Module):
    def __init__(self, vocab: int, d_out: int, mode: Literal["logits", "probs"] = "logits"):
        super().__init__()
        self.vocab, self.mode = vocab, mode
        self.proj = nn.Linear(vocab, d_out, bias=False)

    def forward(self, dist: torch.Tensor) -> torch.Tensor:
        if self.mode == "logits":
            return FN.TextEmbedFn.apply(dist.float(), self.proj.weight)
        return FN.linear(dist, self.proj.weight, None)


class TextProjector(nn.Module):
    def __init__(self, d_in: int, d_proj: int, hidden: int = 0):
        super().__init__()
        self.proj = MLP(d_in, d_proj, hidden)

    def forward(self, z_text: torch.Tensor) -> torch.Tensor:
        return self.proj(z_text)
