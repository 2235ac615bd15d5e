"""Frozen WavLM encoder (forward only) on libfddm_hip.

Parameter tree and state_dict names are those of transformers' WavLMModel (post-LN "group"
geometry, HF modeling_wavlm.py:37-1088), so HF checkpoints of that family load with
load_state_dict. The forward is a fixed kernel sequence per utterance batch:
  conv0+GroupNorm+GELU -> 6 x implicit-GEMM conv+GELU -> LN -> Linear -> grouped positional
  implicit-GEMM conv+GELU -> +x -> LN -> 12 x [gate, QKV GEMM, rel-bias flash attention, out GEMM,
  +x LN, FF GEMM(GELU), FF GEMM, +x LN]
All activations are channels-last [B, T, C] in the compute dtype.
"""
from __future__ import annotations

import json
import os
from types import SimpleNamespace

import torch
import torch.nn as nn

from fddm_hip import ops
from fddm_hip import runtime as rt

# where the bf16 encoder's attention gate comes from (HF modeling_wavlm.py:177-186): "x" (default) the attention
# kernel computes it from the attention input with the folded gru_rel_pos_linear weights; "cols" 8*H extra Q|K|V
# output columns (round 2-5; at the 192-CU encoder cap 2400 columns take 4 tile rounds instead of 3); "separate" the
# fddm_wavlm_gate pass (the fp32 path's)
GATE_MODE = os.environ.get("FDDM_WAVLM_GATE", "x")


def _fold_gate(lin):
    """gru_rel_pos_linear (8 x 64) folded for the in-kernel gate: the reference sums pre-activations 0-3 and 4-7
    (HF modeling_wavlm.py:181-183), so [sum of weight rows 0-3 | rows 4-7 | bias sum 0-3, 4-7] (130 floats)."""
    w, b = lin.weight.detach().float(), lin.bias.detach().float()
    return torch.cat([w[:4].sum(0), w[4:].sum(0), b[:4].sum().reshape(1), b[4:].sum().reshape(1)]).contiguous()

WAVLM_BASE = dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072,
                  conv_dim=(512,) * 7, conv_kernel=(10, 3, 3, 3, 3, 2, 2), conv_stride=(5, 2, 2, 2, 2, 2, 2),
                  conv_bias=False, num_conv_pos_embeddings=128, num_conv_pos_embedding_groups=16, num_buckets=320,
                  max_bucket_distance=800, layer_norm_eps=1e-5, feat_extract_norm="group", do_stable_layer_norm=False,
                  mask_time_prob=0.05, hidden_act="gelu", feat_extract_activation="gelu")


def wavlm_config(**over) -> SimpleNamespace:
    cfg = dict(WAVLM_BASE)
    cfg.update({k: v for k, v in over.items() if k in WAVLM_BASE or k in ("mask_feature_prob",)})
    return SimpleNamespace(**cfg)


class _Sub(nn.Module):
    pass


class WavLMModel(nn.Module):
    def __init__(self, config: SimpleNamespace):
        super().__init__()
        c = config
        if c.feat_extract_norm != "group" or c.do_stable_layer_norm or c.conv_bias:
            raise NotImplementedError("only the post-LN 'group' WavLM geometry (WavLM-base family) is built")
        if c.hidden_size // c.num_attention_heads != 64:
            raise NotImplementedError("head_dim must be 64")
        self.config = c
        fe = _Sub()
        fe.conv_layers = nn.ModuleList()
        cin = 1
        for i, (co, k, s) in enumerate(zip(c.conv_dim, c.conv_kernel, c.conv_stride)):
            layer = _Sub()
            layer.conv = nn.Conv1d(cin, co, kernel_size=k, stride=s, bias=False)
            if i == 0:
                layer.layer_norm = nn.GroupNorm(co, co, affine=True)
            fe.conv_layers.append(layer)
            cin = co
        self.feature_extractor = fe
        fp = _Sub()
        fp.layer_norm = nn.LayerNorm(c.conv_dim[-1], eps=c.layer_norm_eps)
        fp.projection = nn.Linear(c.conv_dim[-1], c.hidden_size)
        self.feature_projection = fp
        if c.mask_time_prob > 0.0:
            self.masked_spec_embed = nn.Parameter(torch.zeros(c.hidden_size).uniform_())
        enc = _Sub()
        pce = _Sub()
        conv = nn.Conv1d(c.hidden_size, c.hidden_size, kernel_size=c.num_conv_pos_embeddings,
                         padding=c.num_conv_pos_embeddings // 2, groups=c.num_conv_pos_embedding_groups)
        pce.conv = nn.utils.parametrizations.weight_norm(conv, name="weight", dim=2)
        enc.pos_conv_embed = pce
        enc.layer_norm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        enc.layers = nn.ModuleList()
        E, H = c.hidden_size, c.num_attention_heads
        for i in range(c.num_hidden_layers):
            L = _Sub()
            a = _Sub()
            a.k_proj, a.v_proj, a.q_proj, a.out_proj = (nn.Linear(E, E) for _ in range(4))
            a.gru_rel_pos_const = nn.Parameter(torch.ones(1, H, 1, 1))
            a.gru_rel_pos_linear = nn.Linear(E // H, 8)
            if i == 0:
                a.rel_attn_embed = nn.Embedding(c.num_buckets, H)
            L.attention = a
            L.layer_norm = nn.LayerNorm(E, eps=c.layer_norm_eps)
            ff = _Sub()
            ff.intermediate_dense = nn.Linear(E, c.intermediate_size)
            ff.output_dense = nn.Linear(c.intermediate_size, E)
            L.feed_forward = ff
            L.final_layer_norm = nn.LayerNorm(E, eps=c.layer_norm_eps)
            enc.layers.append(L)
        self.encoder = enc
        self._prep_key = None
        self._prep = None
        self._plist = None
        self._gen = 0

    # ------------------------------------------------------------------ prepared (cast/permuted) weights
    def _apply(self, fn, *a, **k):     # .to() / .cuda() / .half(): new storage -> re-prepare
        self._gen += 1
        self._plist = None
        return super()._apply(fn, *a, **k)

    def _load_from_state_dict(self, *a, **k):
        self._gen += 1
        return super()._load_from_state_dict(*a, **k)

    def _prepared(self, cd):
        # the encoder is frozen: its prepared (cast / permuted) weights are rebuilt when the module is moved or
        # loaded (_gen) or a parameter is changed in place (the versions, summed over a cached parameter list)
        if self._plist is None:
            self._plist = list(self.parameters())
        key = (cd, self._gen, sum(p._version for p in self._plist))
        if self._prep_key == key:
            return self._prep
        c = self.config
        P = {}
        with torch.no_grad():
            def T(x):
                x = x.detach().contiguous()
                return x if x.dtype == cd else ops.cast(x.float().contiguous(), cd)

            cl = self.feature_extractor.conv_layers
            P["w0"] = cl[0].conv.weight.detach().float().reshape(c.conv_dim[0], -1).contiguous()
            P["gn"] = (cl[0].layer_norm.weight.detach().float().contiguous(), cl[0].layer_norm.bias.detach().float().contiguous())
            P["conv"] = [T(cl[i].conv.weight.permute(0, 2, 1)) for i in range(1, len(cl))]
            fp = self.feature_projection
            P["fp_ln"] = (fp.layer_norm.weight.detach().float(), fp.layer_norm.bias.detach().float())
            P["fp"] = (T(fp.projection.weight), fp.projection.bias.detach().float())
            pc = self.encoder.pos_conv_embed.conv
            w = pc.weight.detach()                                   # weight-norm applied [E, E/G, k]
            G = c.num_conv_pos_embedding_groups
            E = c.hidden_size
            Cg = E // G
            P["pos"] = (T(w.view(G, Cg, Cg, -1).permute(0, 1, 3, 2)), pc.bias.detach().float().contiguous())
            P["enc_ln"] = (self.encoder.layer_norm.weight.detach().float(), self.encoder.layer_norm.bias.detach().float())
            layers = []
            H = c.num_attention_heads
            for L in self.encoder.layers:
                a = L.attention
                qkv_w = [a.q_proj.weight, a.k_proj.weight, a.v_proj.weight]
                qkv_b = [a.q_proj.bias, a.k_proj.bias, a.v_proj.bias]
                if cd == torch.bfloat16 and GATE_MODE == "cols":
                    # gate pre-activations of every head as 8*H extra output columns (block-diagonal copies of
                    # gru_rel_pos_linear), consumed by the attention kernel (no separate gate pass)
                    gw = a.gru_rel_pos_linear.weight.detach().float()
                    blk = torch.zeros(8 * H, E, device=gw.device, dtype=torch.float32)
                    for h in range(H):
                        blk[8 * h:8 * h + 8, h * (E // H):(h + 1) * (E // H)] = gw
                    qkv_w = qkv_w + [blk]
                    qkv_b = qkv_b + [a.gru_rel_pos_linear.bias.detach().float().repeat(H)]
                layers.append(dict(
                    qkv=T(torch.cat([w.detach().float() for w in qkv_w], 0)),
                    bqkv=torch.cat([b.detach().float() for b in qkv_b], 0).contiguous(),
                    o=(T(a.out_proj.weight), a.out_proj.bias.detach().float()),
                    gru=(a.gru_rel_pos_linear.weight.detach().float().contiguous(),
                         a.gru_rel_pos_linear.bias.detach().float().contiguous(),
                         a.gru_rel_pos_const.detach().float().reshape(-1).contiguous()),
                    gw=_fold_gate(a.gru_rel_pos_linear),
                    ln1=(L.layer_norm.weight.detach().float(), L.layer_norm.bias.detach().float()),
                    f1=(T(L.feed_forward.intermediate_dense.weight), L.feed_forward.intermediate_dense.bias.detach().float()),
                    f2=(T(L.feed_forward.output_dense.weight), L.feed_forward.output_dense.bias.detach().float()),
                    ln2=(L.final_layer_norm.weight.detach().float(), L.final_layer_norm.bias.detach().float()),
                ))
            P["layers"] = layers
        self._prep_key, self._prep = key, P
        return P

    def frames(self, nsamp: int) -> int:
        T = nsamp
        for k, s in zip(self.config.conv_kernel, self.config.conv_stride):
            T = (T - k) // s + 1
        return T

    # The forward in three stages (the conv-layer-1 launch on its own, so a HIP-graph replay of the other two keeps
    # the benchmark's probe of that dominant launch an ordinary timed launch: fddm_hip/graphs.py)
    @torch.no_grad()
    def stage_conv0(self, wave: torch.Tensor) -> torch.Tensor:
        """conv layer 0 + GroupNorm + GELU (HF:723-744) -> [B, T0, C] compute dtype."""
        c = self.config
        cd = rt.compute_dtype()
        P = self._prepared(cd)
        wave = wave.float().contiguous()
        return ops.conv0_gn_gelu(wave, P["w0"], P["gn"][0], P["gn"][1], cd, c.conv_dim[0], c.conv_kernel[0],
                                 c.conv_stride[0])

    def conv_out_shape(self, h):
        c = self.config
        B, T, _ = h.shape
        return B, (T - c.conv_kernel[1]) // c.conv_stride[1] + 1, c.conv_dim[1]

    @torch.no_grad()
    def stage_conv1(self, h: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """conv layer 1 + GELU as an implicit GEMM (HF:747-782), the step's largest MFMA launch."""
        return self._conv(h, 1, out)

    def _conv(self, h, i, out=None):
        c = self.config
        P = self._prepared(rt.compute_dtype())
        # persistent-GEMM workgroup cap for the conv layers (train._encoded); layers 2.. may take another
        cap = getattr(self, "conv_cus", 0) if i == 1 else getattr(self, "conv_cus_rest", getattr(self, "conv_cus", 0))
        if cap:
            from fddm_hip._lib import lib
            prev = lib().fddm_gemm_persistent_cap(cap)
            try:
                return self._conv_launch(h, i, out, c, P)
            finally:
                lib().fddm_gemm_persistent_cap(prev)
        return self._conv_launch(h, i, out, c, P)

    def _conv_launch(self, h, i, out, c, P):
        B, T, cin = h.shape
        k, s, co = c.conv_kernel[i], c.conv_stride[i], c.conv_dim[i]
        Tout = (T - k) // s + 1
        if out is None:
            out = torch.empty(B, Tout, co, device=h.device, dtype=h.dtype)
        with rt.probe(f"wavlm.conv{i}"):
            ops.conv1d_gemm(h, P["conv"][i - 1], out, lda=cin, sAb=T * cin, Tin=T, Cg=cin, cstride=s, cpad=0, Bn=B,
                            Tout=Tout, N=co, K=k * cin, gelu=True)
        return out

    @torch.no_grad()
    def stage_rest(self, h: torch.Tensor) -> torch.Tensor:
        """conv layers 2..6, feature projection, positional conv, 12 transformer layers -> [B, S, E]."""
        c = self.config
        cd = rt.compute_dtype()
        P = self._prepared(cd)
        for i in range(2, len(c.conv_dim)):
            h = self._conv(h, i)
        B, T, cin = h.shape
        S, E, H = T, c.hidden_size, c.num_attention_heads
        eps = c.layer_norm_eps
        dev = h.device
        # feature projection (HF:93-105)
        h2 = h.view(B * S, cin)
        hn = torch.empty_like(h2)
        ops.ln_fwd(h2, None, P["fp_ln"][0], P["fp_ln"][1], out_t=hn, eps=eps)
        x = ops.linear(hn, P["fp"][0], P["fp"][1], out_dtype=cd)
        # positional conv embedding + LN (HF:37-90, 399-407)
        G = c.num_conv_pos_embedding_groups
        Cg = E // G
        kp = c.num_conv_pos_embeddings
        pos = torch.empty(B * S, E, device=dev, dtype=cd)
        if cd == torch.bfloat16 and Cg % 16 == 0 and Cg <= 64:
            ops.posconv_gelu(x, P["pos"][0], P["pos"][1], pos, B, S, E, G, kp)   # whole-window LDS kernel
        else:
            ops.conv1d_gemm(x, P["pos"][0], pos, lda=E, sAb=S * E, Tin=S, Cg=Cg, cstride=1, cpad=kp // 2, Bn=B,
                            Tout=S, N=Cg, K=kp * Cg, groups=G, bias=P["pos"][1], gelu=True)
        xn = torch.empty_like(x)
        ops.ln_fwd(x, pos, P["enc_ln"][0], P["enc_ln"][1], out_t=xn, eps=eps)
        x = xn
        table = rt.relbias_table(S, self.encoder.layers[0].attention.rel_attn_embed.weight, c.num_buckets,
                                 c.max_bucket_distance)
        for Lp in P["layers"]:
            qkv = ops.linear(x, Lp["qkv"], Lp["bqkv"], out_dtype=cd)
            o = torch.empty(B * S, E, device=dev, dtype=cd)
            if cd == torch.bfloat16 and GATE_MODE == "x":
                ops.attn_fwd_relgate_x(qkv, qkv[:, E:], qkv[:, 2 * E:], o, x, Lp["gw"], Lp["gru"][2], table, B, H, S)
            elif cd == torch.bfloat16 and GATE_MODE == "cols":
                ops.attn_fwd_relgate(qkv, qkv[:, E:], qkv[:, 2 * E:], o, qkv[:, 3 * E:], Lp["gru"][2], table, B, H, S)
            else:
                gate = ops.wavlm_gate(x, Lp["gru"][0], Lp["gru"][1], Lp["gru"][2], B, S, H)
                ops.attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], o, None, B, H, S, S, gate=gate, table=table)
            y = ops.linear(o, Lp["o"][0], Lp["o"][1], out_dtype=cd)
            x1 = torch.empty_like(x)
            ops.ln_fwd(x, y, Lp["ln1"][0], Lp["ln1"][1], out_t=x1, eps=eps)
            hh = ops.linear(x1, Lp["f1"][0], Lp["f1"][1], out_dtype=cd, epi=ops.EPI_GELU_ONLY)
            y = ops.linear(hh, Lp["f2"][0], Lp["f2"][1], out_dtype=cd)
            x = torch.empty_like(x1)
            ops.ln_fwd(x1, y, Lp["ln2"][0], Lp["ln2"][1], out_t=x, eps=eps)
        return x.view(B, S, E)

    @torch.no_grad()
    def forward_hidden(self, wave: torch.Tensor) -> torch.Tensor:
        """last_hidden_state [B, S, E] in the compute dtype (eval mode, attention_mask=None)."""
        return self.stage_rest(self.stage_conv1(self.stage_conv0(wave)))

    def forward(self, input_values, attention_mask=None, output_hidden_states=False, **kw):
        if attention_mask is not None:
            raise NotImplementedError("attention_mask is never passed on the train step (lengths=None)")
        return SimpleNamespace(last_hidden_state=self.forward_hidden(input_values))

    # ------------------------------------------------------------------ loading
    random_init = True      # False once weights were loaded from a checkpoint

    @staticmethod
    def hf_state_dict(sd: dict) -> dict:
        """A transformers WavLM checkpoint's state_dict in this module's names: strips the `wavlm.` prefix of
        task-head checkpoints (dropping the heads), and maps the legacy weight-norm names of the positional conv
        (`weight_g` / `weight_v`, torch.nn.utils.weight_norm) to the parametrization names
        (`parametrizations.weight.original0/1`, torch.nn.utils.parametrizations.weight_norm) that HF
        modeling_wavlm.py:45-66 registers on current torch."""
        if any(k.startswith("wavlm.") for k in sd):
            sd = {k[len("wavlm."):]: v for k, v in sd.items() if k.startswith("wavlm.")}
        out = {}
        for k, v in sd.items():
            if k.endswith("pos_conv_embed.conv.weight_g"):
                k = k[: -len("weight_g")] + "parametrizations.weight.original0"
            elif k.endswith("pos_conv_embed.conv.weight_v"):
                k = k[: -len("weight_v")] + "parametrizations.weight.original1"
            out[k] = v
        return out

    @classmethod
    def from_pretrained(cls, name_or_path, geometry: dict | None = None):
        """Local directory with config.json + model.safetensors / pytorch_model.bin -> loaded weights (strict:
        a missing or unexpected key raises). A dict -> that geometry, random init. Anything else (a hub name;
        there is no network) -> WavLM-base geometry, random init. `random_init` tells the two apart (train.py
        refuses a random-init encoder unless asked to allow it)."""
        if isinstance(name_or_path, dict):
            return cls(wavlm_config(**name_or_path))
        path = str(name_or_path)
        if os.path.isdir(path) and os.path.exists(os.path.join(path, "config.json")):
            cfg = json.load(open(os.path.join(path, "config.json")))
            m = cls(wavlm_config(**cfg))
            sd = None
            st_path = os.path.join(path, "model.safetensors")
            bin_path = os.path.join(path, "pytorch_model.bin")
            if os.path.exists(st_path):
                from safetensors.torch import load_file
                sd = load_file(st_path)
            elif os.path.exists(bin_path):
                sd = torch.load(bin_path, map_location="cpu", weights_only=True)
            if sd is None:
                raise FileNotFoundError(f"{path}: config.json but no model.safetensors / pytorch_model.bin")
            sd = cls.hf_state_dict(sd)
            if "masked_spec_embed" not in sd and hasattr(m, "masked_spec_embed"):
                sd["masked_spec_embed"] = m.masked_spec_embed.detach().clone()   # unused in eval (HF:1006)
            missing, unexpected = m.load_state_dict(sd, strict=False)
            if missing or unexpected:
                raise RuntimeError(f"{path}: WavLM checkpoint does not match the geometry: missing {missing[:8]}, "
                                   f"unexpected {unexpected[:8]}")
            m.random_init = False
            return m
        return cls(wavlm_config(**(geometry or {})))
