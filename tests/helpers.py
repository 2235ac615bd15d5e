"""Shared test helpers: PCG parameter dicts with reference names, fixture loading, comparisons."""
import os

import numpy as np
import torch

from conftest import GOLDEN
from oracle.weights import pcg_array


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def T(a):
    return torch.from_numpy(np.asarray(a))


def close(a, b, rtol=1e-5, atol=1e-6, what=""):
    a = a.detach().double().cpu() if torch.is_tensor(a) else torch.tensor(a, dtype=torch.float64)
    b = T(b).double() if not torch.is_tensor(b) else b.detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    assert torch.isfinite(a).all(), f"{what}: non-finite values"
    err = (a - b).abs().max().item() if a.numel() else 0.0
    tol = atol + rtol * b.abs().max().item() if b.numel() else atol
    assert err <= tol, f"{what}: max err {err:.3e} > tol {tol:.3e} (ref max {b.abs().max().item():.3e})"


def _dec_sd(V, d, H, NL, FF, prefix="dec."):
    from oracle.weights import pcg_array as P

    shapes = {"tok_emb.weight": (V, d), "time_emb.mlp.0.weight": (4 * d, d), "time_emb.mlp.0.bias": (4 * d,),
              "time_emb.mlp.2.weight": (d, 4 * d), "time_emb.mlp.2.bias": (d,), "time_proj.weight": (d, d),
              "time_proj.bias": (d,), "head.weight": (V, d), "head.bias": (V,)}
    for i in range(NL):
        b = f"blocks.{i}."
        for a in ("self_attn.", "cross_attn."):
            shapes[b + a + "in_proj_weight"] = (3 * d, d)
            shapes[b + a + "in_proj_bias"] = (3 * d,)
            shapes[b + a + "out_proj.weight"] = (d, d)
            shapes[b + a + "out_proj.bias"] = (d,)
        for f in ("scale_proj.", "shift_proj."):
            shapes[b + "film_layer." + f + "weight"] = (d, d)
            shapes[b + "film_layer." + f + "bias"] = (d,)
        shapes[b + "ff.0.weight"] = (FF, d)
        shapes[b + "ff.0.bias"] = (FF,)
        shapes[b + "ff.3.weight"] = (d, FF)
        shapes[b + "ff.3.bias"] = (d,)
        for n in ("norm1.", "norm2.", "norm3."):
            shapes[b + n + "weight"] = (d,)
            shapes[b + n + "bias"] = (d,)
    sd = {n: T(P(prefix + n, s)) for n, s in shapes.items()}
    sd["tok_emb.weight"][0] = 0.0
    return sd


SMALL_WAVLM = dict(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=256,
                   conv_dim=(32,) * 7, num_conv_pos_embedding_groups=4)


def wavlm_sd(geom, d_model, with_proj=True):
    E = geom["hidden_size"]
    C = geom["conv_dim"]
    H = geom["num_attention_heads"]
    shapes = {}
    cin = 1
    for i, (c, k) in enumerate(zip(C, geom["conv_kernel"])):
        shapes[f"backbone.feature_extractor.conv_layers.{i}.conv.weight"] = (c, cin, k)
        cin = c
    shapes["backbone.feature_extractor.conv_layers.0.layer_norm.weight"] = (C[0],)
    shapes["backbone.feature_extractor.conv_layers.0.layer_norm.bias"] = (C[0],)
    shapes["backbone.feature_projection.layer_norm.weight"] = (C[-1],)
    shapes["backbone.feature_projection.layer_norm.bias"] = (C[-1],)
    shapes["backbone.feature_projection.projection.weight"] = (E, C[-1])
    shapes["backbone.feature_projection.projection.bias"] = (E,)
    kp, gp = geom["num_conv_pos_embeddings"], geom["num_conv_pos_embedding_groups"]
    shapes["backbone.encoder.pos_conv_embed.conv.bias"] = (E,)
    shapes["backbone.encoder.pos_conv_embed.conv.parametrizations.weight.original0"] = (1, 1, kp)
    shapes["backbone.encoder.pos_conv_embed.conv.parametrizations.weight.original1"] = (E, E // gp, kp)
    shapes["backbone.encoder.layer_norm.weight"] = (E,)
    shapes["backbone.encoder.layer_norm.bias"] = (E,)
    for i in range(geom["num_hidden_layers"]):
        p = f"backbone.encoder.layers.{i}."
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            shapes[p + f"attention.{n}.weight"] = (E, E)
            shapes[p + f"attention.{n}.bias"] = (E,)
        shapes[p + "attention.gru_rel_pos_const"] = (1, H, 1, 1)
        shapes[p + "attention.gru_rel_pos_linear.weight"] = (8, E // H)
        shapes[p + "attention.gru_rel_pos_linear.bias"] = (8,)
        if i == 0:
            shapes[p + "attention.rel_attn_embed.weight"] = (geom["num_buckets"], H)
        shapes[p + "layer_norm.weight"] = (E,)
        shapes[p + "layer_norm.bias"] = (E,)
        shapes[p + "feed_forward.intermediate_dense.weight"] = (geom["intermediate_size"], E)
        shapes[p + "feed_forward.intermediate_dense.bias"] = (geom["intermediate_size"],)
        shapes[p + "feed_forward.output_dense.weight"] = (E, geom["intermediate_size"])
        shapes[p + "feed_forward.output_dense.bias"] = (E,)
        shapes[p + "final_layer_norm.weight"] = (E,)
        shapes[p + "final_layer_norm.bias"] = (E,)
    if with_proj and E != d_model:
        shapes["proj.weight"] = (d_model, E)
        shapes["proj.bias"] = (d_model,)
    return {n: T(pcg_array(n, s)) for n, s in shapes.items()}


def _step_params(V, d, NL, FF, H):
    sd = _dec_sd(V, d, H, NL, FF)
    params = {"decoder." + n: p for n, p in sd.items()}
    params["s_proj.proj.net.0.weight"] = T(pcg_array("s_proj.proj.net.0.weight", (256, d)))
    params["s_proj.proj.net.0.bias"] = T(pcg_array("s_proj.proj.net.0.bias", (256,)))
    params["t_embed.proj.weight"] = T(pcg_array("t_embed.proj.weight", (256, V)))
    params["t_proj.proj.net.0.weight"] = T(pcg_array("t_proj.proj.net.0.weight", (256, 256)))
    params["t_proj.proj.net.0.bias"] = T(pcg_array("t_proj.proj.net.0.bias", (256,)))
    return params




def jumpy_case_inputs(i, B, L, K):
    """Seeded inputs of jumpy posterior case i — the same numpy-PCG64 draws as
    tests/golden/make_golden.py:jumpy_case_inputs (the fixture stores only the outputs)."""
    r = np.random.Generator(np.random.PCG64(300 + i))
    logits = torch.from_numpy(3.0 * r.standard_normal((B, L, K), dtype=np.float32))
    xt = torch.from_numpy(r.integers(0, K, size=(B, L))).long()
    boost = torch.from_numpy(r.uniform(-10.0, 6.0, size=(B, L)).astype(np.float32))
    logits.scatter_add_(-1, xt[..., None], boost[..., None])
    return logits, xt


class CollectiveLog:
    """Records every torch.distributed collective issued inside the context (name, shape, dtype, reduce op), in
    issue order: DP ranks must issue the identical sequence (fddm_hip.dist, train.train_one_epoch)."""

    NAMES = ("all_reduce", "broadcast", "all_gather", "all_gather_into_tensor", "reduce_scatter_tensor",
             "all_gather_object", "barrier")

    def __init__(self):
        self.log = []
        self._orig = {}

    def __enter__(self):
        import torch.distributed as dist
        for n in self.NAMES:
            f = getattr(dist, n, None)
            if f is None:
                continue
            self._orig[n] = f

            def wrap(*a, _n=n, _f=f, **k):
                t = a[0] if a and hasattr(a[0], "shape") else None
                op = k.get("op", a[1] if _n == "all_reduce" and len(a) > 1 else None)
                self.log.append((_n, tuple(t.shape) if t is not None else None, str(t.dtype) if t is not None
                                 else None, str(op) if op is not None else None))
                return _f(*a, **k)
            setattr(dist, n, wrap)
        return self

    def __exit__(self, *exc):
        import torch.distributed as dist
        for n, f in self._orig.items():
            setattr(dist, n, f)
        return False
