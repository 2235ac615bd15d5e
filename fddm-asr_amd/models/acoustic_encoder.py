"""AcousticEncoder (drop-in for models/acoustic_encoder.py of the reference, lines 34-128).

Same constructor and forward contract: forward(waveforms[B,T], lengths=None) ->
(features [B,S,d_model], feat_mask or None, pooled or None); attributes backbone / proj / use_proj /
pooling; state_dict keys `backbone.<HF WavLM names>` and `proj.*`.

`wavlm_name` may be a local HF-format directory (loaded), a dict of WavLMConfig geometry overrides,
or a hub name (no network here: WavLM-base geometry with random init, as the benchmark specifies).
The encoder is frozen and runs forward-only on libfddm_hip; its output is returned without autograd
history (the reference's encoder.proj receives a gradient it never applies, train.py:543).
"""
from __future__ import annotations

import logging
from typing import Optional, Tuple

import torch
import torch.nn as nn

from fddm_hip import functions as FN
from fddm_hip import ops
from fddm_hip import runtime as rt

from .wavlm import WavLMModel


class AcousticEncoder(nn.Module):
    def __init__(self, wavlm_name="microsoft/wavlm-large", freeze: bool = True, d_model: int = 768,
                 proj: str = "linear", pooling: str = "none") -> None:
        super().__init__()
        if isinstance(wavlm_name, str) and not wavlm_name.startswith("/") and not wavlm_name.startswith("."):
            logging.getLogger(__name__).warning(
                "AcousticEncoder: %r is a hub name; no network -> WavLM-base geometry, random init", wavlm_name)
        self.backbone = WavLMModel.from_pretrained(wavlm_name)
        hidden = self.backbone.config.hidden_size
        if freeze:
            for p in self.backbone.parameters():
                p.requires_grad_(False)
        self.use_proj = (proj == "linear") and (hidden != d_model)
        self.proj = nn.Linear(hidden, d_model) if self.use_proj else nn.Identity()
        assert pooling in {"none", "mean"}
        self.pooling = pooling

    @torch.no_grad()
    def _make_mask(self, lengths: torch.Tensor, max_len: int) -> torch.Tensor:
        ids = torch.arange(max_len, device=lengths.device).unsqueeze(0)
        return ids < lengths.unsqueeze(1)

    def forward(self, waveforms: torch.Tensor, lengths: Optional[torch.Tensor] = None
                ) -> Tuple[torch.Tensor, Optional[torch.Tensor], Optional[torch.Tensor]]:
        if lengths is not None:
            raise NotImplementedError("lengths-masked encoding is not on the train step (train.py:349)")
        with torch.no_grad():
            feats = self.project(self.backbone.forward_hidden(waveforms))
        pooled = feats.float().mean(dim=1) if self.pooling == "mean" else None
        return feats, None, pooled

    @torch.no_grad()
    def project(self, h: torch.Tensor) -> torch.Tensor:
        """encoder.proj (acoustic_encoder.py:107) on the backbone's [B, S, hidden] output (identity if hidden ==
        d_model)."""
        if not self.use_proj:
            return h
        B, S, E = h.shape
        cd = rt.compute_dtype()
        return ops.linear(h.view(B * S, E), rt.wt(self.proj.weight), self.proj.bias.detach(),
                          out_dtype=cd).view(B, S, -1)
