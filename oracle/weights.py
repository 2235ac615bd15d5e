"""Deterministic parameter generator shared by the golden-vector script and the tests.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Every parameter of a module is drawn from
numpy PCG64 seeded by (seed, crc32(name)), so the golden generator (which runs the reference here)
and the GPU-box tests (which never see the reference) build bit-identical weights from names alone.
"""
from __future__ import annotations

import math
import zlib

import numpy as np
import torch


def pcg_array(name: str, shape, seed: int = 1234) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    rng = np.random.Generator(np.random.PCG64([int(seed), zlib.crc32(name.encode())]))
    x = rng.standard_normal(shape, dtype=np.float32) if shape else rng.standard_normal(dtype=np.float32)
    x = np.asarray(x, dtype=np.float32)
    leaf = name.rsplit(".", 1)[-1]
    is_norm = ("norm" in name) and len(shape) == 1
    if leaf == "gru_rel_pos_const":
        return (1.0 + 0.1 * x).astype(np.float32)
    if leaf == "inv_freq":
        raise ValueError("buffers are not generated")
    if is_norm and leaf == "weight":
        return (1.0 + 0.05 * x).astype(np.float32)
    if leaf == "bias" or len(shape) <= 1:
        return (0.02 * x).astype(np.float32)
    if "rel_attn_embed" in name:
        return (0.5 * x).astype(np.float32)
    if name.endswith("original0"):  # weight-norm magnitude g
        return (0.5 + 0.1 * np.abs(x)).astype(np.float32)
    if "tok_emb" in name:
        return x
    fan_in = int(np.prod(shape[1:]))
    return (x / math.sqrt(fan_in)).astype(np.float32)


def pcg_state_dict(module: torch.nn.Module, seed: int = 1234, prefix: str = "", skip=()) -> dict:
    """Build a full state dict of PCG tensors for `module`'s parameters (buffers are kept)."""
    sd = {}
    pnames = {n for n, _ in module.named_parameters()}
    for n, t in module.state_dict().items():
        if n in pnames and not any(n.startswith(s) for s in skip):
            sd[n] = torch.from_numpy(pcg_array(prefix + n, t.shape, seed)).to(t.dtype)
        else:
            sd[n] = t.clone()
    return sd


def load_pcg(module: torch.nn.Module, seed: int = 1234, prefix: str = "", pad_row=None) -> None:
    sd = pcg_state_dict(module, seed, prefix)
    if pad_row is not None:
        name, idx = pad_row
        if name in sd:
            sd[name][idx] = 0.0
    module.load_state_dict(sd, strict=True)
