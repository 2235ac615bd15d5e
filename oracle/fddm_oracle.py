"""CPU oracle for the FDDM-ASR train step (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Every function restates the reference algorithm in plain fp32 torch on the CPU and cites the
reference lines it follows (paths relative to /root/reference; `HF:` = transformers 5.15.0
models/wavlm/modeling_wavlm.py, the third-party code the reference's encoder calls).
Pinned by tests/test_oracle_golden.py against fixtures produced by the reference itself.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

# ------------------------------------------------------------------------------------------------
# RNG contract (build-defined; the reference uses torch's mt19937 stream, which is not reproducible
# on a GPU). Counter-based splitmix64: value = fin(seed*G + stream*S + idx). The HIP kernels
# implement the identical integer arithmetic (csrc/common.h: fddm_mix), so integer outputs
# (sampled token ids, dropout masks) are bit-exact between GPU and this oracle.
# ------------------------------------------------------------------------------------------------
_G = np.uint64(0x9E3779B97F4A7C15)
_S = np.uint64(0xD1B54A32D192ED03)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def mix64(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) * _G + np.uint64(stream) * _S + idx.astype(np.uint64)
        z = z + _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def dropout_keep(seed: int, stream: int, numel: int, p: float) -> torch.Tensor:
    """Keep-mask for `numel` elements: element e keeps iff u16(e) >= round(p*65536), where
    u16(e) = bits [16*(e&3), 16*(e&3)+16) of mix64(seed, stream, e>>2)."""
    e = np.arange(numel, dtype=np.uint64)
    h = mix64(seed, stream, e >> np.uint64(2))
    u = (h >> (np.uint64(16) * (e & np.uint64(3)))) & np.uint64(0xFFFF)
    thr = int(round(p * 65536.0))
    return torch.from_numpy(u >= np.uint64(thr))


ATTN_R = 4096
_ATTN_TAB0 = np.uint64(1 << 62)
_ATTN_OFF0 = np.uint64(3 << 62)


def attn_dropout_keep(seed: int, stream: int, B: int, H: int, Lq: int, Lk: int, p: float) -> torch.Tensor:
    """Keep-mask [B, H, Lq, Lk] of the attention-probability dropout (RNG contract v2, the dropout on
    softmax(QK^T) inside nn.MultiheadAttention, models/denoise_decoder.py:129-130; csrc/attention.hip).
    Per (b, h) = bh three tables of R = 4096 16-bit draws, T_tau[j] = bits 16*(j&3).. of
    mix64(seed, stream, 2^62 + (bh*3 + tau)*1024 + (j>>2)); per query row r = bh*Lq + q three offsets
    o_tau = (mix64(seed, stream, 3*2^62 + r) >> 16*tau) & 0xFFC; element (q, k) keeps iff
    T_0[(o_0+k)%R] ^ T_1[(o_1+k)%R] ^ T_2[(o_2+k)%R] >= round(p*65536)."""
    thr = int(round(p * 65536.0))
    BH = B * H
    words = mix64(seed, stream, _ATTN_TAB0 + np.arange(BH * 3 * (ATTN_R // 4), dtype=np.uint64))
    shifts = (np.uint64(16) * np.arange(4, dtype=np.uint64))
    tab = ((words[:, None] >> shifts[None, :]) & np.uint64(0xFFFF)).reshape(BH, 3, ATTN_R)     # [BH, 3, R]
    rows = np.arange(BH * Lq, dtype=np.uint64)
    off = mix64(seed, stream, _ATTN_OFF0 + rows).reshape(BH, Lq)
    k = np.arange(Lk, dtype=np.int64)
    u = np.zeros((BH, Lq, Lk), dtype=np.uint64)
    for tau in range(3):
        o = ((off >> np.uint64(16 * tau)) & np.uint64(0xFFC)).astype(np.int64)                  # [BH, Lq]
        j = (o[:, :, None] + k[None, None, :]) % ATTN_R
        u ^= np.take_along_axis(tab[:, tau, :], j.reshape(BH, -1), axis=1).reshape(BH, Lq, Lk)
    return torch.from_numpy(u >= np.uint64(thr)).view(B, H, Lq, Lk)


# ------------------------------------------------------------------------------------------------
# Scheduler — fddm/sched/diffusion_scheduler.py:18-29 (cosine betas, cumprod alpha_bar, fp32)
# ------------------------------------------------------------------------------------------------
def sched_tables(T: int, beta_max: float = 0.2):
    t = torch.arange(1, T + 1, dtype=torch.float32)
    betas = beta_max * torch.sin(0.5 * math.pi * (t / float(T))) ** 2
    alpha_bar = torch.cumprod(1.0 - betas, dim=0)
    return betas, alpha_bar


def q_sample_values(K: int, alpha_bar: torch.Tensor, eps: float = 1e-8):
    """q_sample (diffusion_scheduler.py:31-50) produces two distinct probabilities per t: p_hi at
    x0 and p_lo elsewhere (after clamp_min(eps) and renormalisation). Returns (p_hi, p_lo) fp32 [T]."""
    ab = alpha_bar.float()
    u = torch.tensor(1.0 / K, dtype=torch.float32)
    hi = ab * 1.0 + (1.0 - ab) * u
    lo = ab * 0.0 + (1.0 - ab) * u
    hi = hi.clamp_min(eps)
    lo = lo.clamp_min(eps)
    s = (hi + (K - 1) * lo.double()).float()  # row sum of the K entries
    s = s.clamp_min(eps)
    return hi / s, lo / s


def sample_thresholds(K: int, alpha_bar: torch.Tensor) -> np.ndarray:
    """uint32 keep-thresholds per t: P(xt = x0) = p_hi  ->  thr = floor(p_hi * 2^32) (clamped)."""
    hi, _ = q_sample_values(K, alpha_bar)
    thr = np.floor(hi.double().numpy() * 4294967296.0)
    return np.clip(thr, 0, 4294967295).astype(np.uint64)


def sample_xt(x0: torch.Tensor, t: torch.Tensor, K: int, alpha_bar: torch.Tensor, seed: int, stream: int = 1) -> torch.Tensor:
    """Closed-form two-valued inverse CDF for SchedulerAdapter.sample_q (train.py:180-188).
    token (b,l) index e: h = mix64(seed, stream, e); r1 = h>>32 keeps x0 iff r1 < thr[t];
    otherwise j = (r2*(K-1))>>32 with r2 = h & 0xffffffff, and xt = j + (j >= x0)."""
    B, L = x0.shape
    thr = sample_thresholds(K, alpha_bar)
    e = np.arange(B * L, dtype=np.uint64)
    h = mix64(seed, stream, e)
    r1 = h >> np.uint64(32)
    r2 = h & np.uint64(0xFFFFFFFF)
    x0n = x0.reshape(-1).numpy().astype(np.int64)
    tn = np.repeat(t.numpy().astype(np.int64), L)
    keep = r1 < thr[tn - 1]
    with np.errstate(over="ignore"):
        j = ((r2 * np.uint64(K - 1)) >> np.uint64(32)).astype(np.int64)
    other = j + (j >= x0n)
    out = np.where(keep, x0n, other)
    return torch.from_numpy(out.reshape(B, L)).long()


# ------------------------------------------------------------------------------------------------
# KL term — train.py:190-255, closed form (SURVEY §8(a) "KL closed form")
# ------------------------------------------------------------------------------------------------
def kl_term(logits: torch.Tensor, xt: torch.Tensor, x0: torch.Tensor, t: torch.Tensor,
            x_mask: Optional[torch.Tensor], betas: torch.Tensor):
    """Returns (loss, dloss/dlogits) computed from the closed form (fp32)."""
    B, L, V = logits.shape
    eps = 1e-8
    K = float(V)
    z = logits.float()
    xhat = torch.softmax(z, dim=-1)
    bt = betas[t - 1].float().view(B, 1)                                   # train.py:214
    bp = torch.where(t.eq(1), torch.zeros(()), betas[(t - 2).clamp(min=0)]).float().view(B, 1)  # :215-217
    a_t, b_t = 1.0 - bt, bt / K
    a_p, b_p = 1.0 - bp, bp / K
    is_xt = F.one_hot(xt, V).bool()
    is_x0 = F.one_hot(x0, V).bool()
    M = b_t[..., None] + a_t[..., None] * is_xt.float()                    # :227
    d_q = b_t + a_t * (x0 == xt).float()                                     # :238
    xhat_xt = torch.gather(xhat, -1, xt[..., None])[..., 0]
    d_p = b_t + a_t * xhat_xt                                                # :239
    Q = M * (a_p[..., None] * is_x0.float() + b_p[..., None]) / (d_q[..., None] + eps)   # :242
    P = M * (a_p[..., None] * xhat + b_p[..., None]) / (d_p[..., None] + eps)            # :243
    kl_tok = (Q * (torch.log(Q + eps) - torch.log(P + eps))).sum(-1)        # :246
    if x_mask is not None:
        valid = x_mask.float()
        denom = valid.sum(1) + eps
        per = (kl_tok * valid).sum(1) / denom                               # :251
        w = valid / denom[:, None] / B
    else:
        per = kl_tok.mean(1)                                                 # :253
        w = torch.full((B, L), 1.0 / (L * B))
    loss = per.mean()
    # gradient (closed form)
    S1 = (Q * P / (P + eps)).sum(-1)
    g = -Q * M * a_p[..., None] / ((P + eps) * (d_p[..., None] + eps))
    g = g + is_xt.float() * (a_t * S1 / (d_p + eps))[..., None]
    dz = w[..., None] * xhat * (g - (g * xhat).sum(-1, keepdim=True))
    return loss, dz


# ------------------------------------------------------------------------------------------------
# RoPE — models/denoise_decoder.py:25-53
# ------------------------------------------------------------------------------------------------
def rope_inv_freq(d: int, base: float = 10000.0) -> torch.Tensor:
    return 1.0 / (base ** (torch.arange(0, d, 2).float() / d))


def rope_cos_sin(L: int, inv_freq: torch.Tensor):
    t = torch.arange(L, dtype=inv_freq.dtype)
    freqs = torch.outer(t, inv_freq)
    emb = torch.cat((freqs, freqs), dim=-1)
    return emb.cos(), emb.sin()


def rope_apply(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    x1, x2 = x[..., ::2], x[..., 1::2]
    return torch.cat([x1 * cos[..., ::2] - x2 * sin[..., 1::2], x1 * sin[..., ::2] + x2 * cos[..., 1::2]], dim=-1)


# ------------------------------------------------------------------------------------------------
# Decoder — models/denoise_decoder.py:92-287 with torch.nn.MultiheadAttention semantics
# ------------------------------------------------------------------------------------------------
def time_embedding(t: torch.Tensor, d: int, max_steps: int = 10000) -> torch.Tensor:
    half = d // 2                                                            # :108-116
    freqs = torch.exp(torch.linspace(math.log(1.0), math.log(max_steps), half) * (-1))
    args = t.float().unsqueeze(1) * freqs.unsqueeze(0)
    emb = torch.cat([torch.sin(args), torch.cos(args)], dim=1)
    if d % 2 == 1:
        emb = F.pad(emb, (0, 1))
    return emb


def mha(q_in, k_in, v_in, W, bias, Wo, bo, H, key_keep=None, drop_p=0.0, drop=None):
    """nn.MultiheadAttention(batch_first) forward (torch F.multi_head_attention_forward, explicit path)."""
    B, Lq, d = q_in.shape
    Lk = k_in.shape[1]
    dh = d // H
    q = F.linear(q_in, W[:d], bias[:d])
    k = F.linear(k_in, W[d:2 * d], bias[d:2 * d])
    v = F.linear(v_in, W[2 * d:], bias[2 * d:])
    q = q.view(B, Lq, H, dh).transpose(1, 2)
    k = k.view(B, Lk, H, dh).transpose(1, 2)
    v = v.view(B, Lk, H, dh).transpose(1, 2)
    s = (q * (1.0 / math.sqrt(dh))) @ k.transpose(-1, -2)
    if key_keep is not None:
        s = s.masked_fill(~key_keep[:, None, None, :], float("-inf"))
    p = torch.softmax(s, -1)
    if drop is not None and drop_p > 0:
        p = drop.attn(p)
    o = (p @ v).transpose(1, 2).reshape(B, Lq, d)
    return F.linear(o, Wo, bo)


_MASKS: dict = {}      # (kind, args) -> keep mask: the contract's masks are pure functions of their arguments


def _memo_mask(key, make):
    m = _MASKS.get(key)
    if m is None:
        if len(_MASKS) >= 96:
            _MASKS.clear()
        m = _MASKS[key] = make()
    return m


class _Dropper:
    """Deterministic dropout per site following the RNG contract (seed, stream = base + site)."""

    def __init__(self, p: float, seed: int):
        self.p, self.seed, self.site = p, seed, 0

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        self.site += 1
        if self.p <= 0:
            return x
        keep = _memo_mask(("e", self.seed, self.site, x.numel(), self.p),
                          lambda: dropout_keep(self.seed, self.site, x.numel(), self.p)).view(x.shape)
        return x * keep.float() * (1.0 / (1.0 - self.p))

    def attn(self, p: torch.Tensor) -> torch.Tensor:
        """Attention-probability site (p [B, H, Lq, Lk]): RNG contract v2 (attn_dropout_keep)."""
        self.site += 1
        if self.p <= 0:
            return p
        B, H, Lq, Lk = p.shape
        keep = _memo_mask(("a", self.seed, self.site, B, H, Lq, Lk, self.p),
                          lambda: attn_dropout_keep(self.seed, self.site, B, H, Lq, Lk, self.p))
        return p * keep.to(p.dtype) * (1.0 / (1.0 - self.p))


def decoder_block(sd, pre, x, cond, x_mask, cos, sin, H, drop: Optional[_Dropper] = None, c_mask=None):
    """DecoderBlock.forward — models/denoise_decoder.py:147-192."""
    p = drop.p if drop is not None else 0.0
    D = (lambda z: drop(z)) if drop is not None else (lambda z: z)
    d = x.shape[-1]
    qk = rope_apply(x, cos, sin)                                             # :157-159
    a = pre + "self_attn."
    x2 = mha(qk, qk, x, sd[a + "in_proj_weight"], sd[a + "in_proj_bias"], sd[a + "out_proj.weight"],
             sd[a + "out_proj.bias"], H, key_keep=x_mask, drop_p=p, drop=drop)   # :164
    x = F.layer_norm(x + D(x2), (d,), sd[pre + "norm1.weight"], sd[pre + "norm1.bias"], 1e-5)   # :165-166
    a = pre + "cross_attn."
    x2 = mha(x, cond, cond, sd[a + "in_proj_weight"], sd[a + "in_proj_bias"], sd[a + "out_proj.weight"],
             sd[a + "out_proj.bias"], H, key_keep=c_mask, drop_p=p, drop=drop)  # :169-174
    x = F.layer_norm(x + D(x2), (d,), sd[pre + "norm2.weight"], sd[pre + "norm2.bias"], 1e-5)   # :175-176
    pooled = cond.mean(dim=1)                                                # :185
    scale = F.linear(pooled, sd[pre + "film_layer.scale_proj.weight"], sd[pre + "film_layer.scale_proj.bias"])
    shift = F.linear(pooled, sd[pre + "film_layer.shift_proj.weight"], sd[pre + "film_layer.shift_proj.bias"])
    x = x * (1 + scale[:, None]) + shift[:, None]                            # :87-89
    h = F.gelu(F.linear(x, sd[pre + "ff.0.weight"], sd[pre + "ff.0.bias"]))  # :136-141
    h = D(h)
    x2 = F.linear(h, sd[pre + "ff.3.weight"], sd[pre + "ff.3.bias"])
    x = F.layer_norm(x + D(x2), (d,), sd[pre + "norm3.weight"], sd[pre + "norm3.bias"], 1e-5)   # :189-191
    return x


def decoder_forward(sd: Dict[str, torch.Tensor], xt, t, cond, x_mask, H: int, num_layers: int, pad_id: int = 0,
                    dropout: float = 0.0, seed: int = 0, taps: Optional[list] = None):
    """DenoisingTransformerDecoder.forward — models/denoise_decoder.py:242-287. `taps` (a list, optional) receives
    each block's output x (with retain_grad() when it requires grad), for per-block error budgets in tests."""
    d = sd["tok_emb.weight"].shape[1]
    L = xt.shape[1]
    x = F.embedding(xt, sd["tok_emb.weight"], padding_idx=pad_id)            # :254
    inv_freq = rope_inv_freq(d)
    cos, sin = rope_cos_sin(L, inv_freq)                                     # :260
    te = time_embedding(t, d)
    te = F.linear(F.silu(F.linear(te, sd["time_emb.mlp.0.weight"], sd["time_emb.mlp.0.bias"])),
                  sd["time_emb.mlp.2.weight"], sd["time_emb.mlp.2.bias"])
    x = x + F.linear(te, sd["time_proj.weight"], sd["time_proj.bias"])[:, None]   # :272-274
    if x_mask is None:
        x_mask = xt != pad_id                                                # :277-278
    drop = _Dropper(dropout, seed) if dropout > 0 else None
    for i in range(num_layers):
        x = decoder_block(sd, f"blocks.{i}.", x, cond, x_mask, cos, sin, H, drop)
        if taps is not None:
            if x.requires_grad:
                x.retain_grad()
            taps.append(x)
    return F.linear(x, sd["head.weight"], sd["head.bias"])                    # :286


# ------------------------------------------------------------------------------------------------
# L_fd — losses/fddm_losses.py:18-58
# ------------------------------------------------------------------------------------------------
def lfd_loss(z_a, z_b, lambda_offdiag=5e-3, eps=1e-5):
    B, T, D = z_a.shape

    def std(x):
        m = x.mean(0, keepdim=True)
        v = x.var(0, unbiased=False, keepdim=True)
        return (x - m) / torch.sqrt(v + eps)

    za, zb = std(z_a).reshape(B * T, D), std(z_b).reshape(B * T, D)
    Cm = za.T @ zb / (B * T)
    diag = torch.diagonal(Cm)
    off = Cm - torch.diag(diag)
    return ((1.0 - diag) ** 2).sum() + lambda_offdiag * (off ** 2).sum()


def align_speech(z_speech: torch.Tensor, L: int) -> torch.Tensor:
    """S->L alignment — train.py:382-387."""
    S = z_speech.shape[1]
    if S >= L:
        return z_speech[:, :L]
    return torch.cat([z_speech, z_speech[:, -1:].repeat(1, L - S, 1)], dim=1)


# ------------------------------------------------------------------------------------------------
# WavLM encoder — HF modeling_wavlm.py (forward, eval mode, post-LN "group" geometry)
# ------------------------------------------------------------------------------------------------
WAVLM_BASE = dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072,
                  conv_dim=(512,) * 7, conv_kernel=(10, 3, 3, 3, 3, 2, 2), conv_stride=(5, 2, 2, 2, 2, 2, 2),
                  num_conv_pos_embeddings=128, num_conv_pos_embedding_groups=16, num_buckets=320,
                  max_bucket_distance=800, layer_norm_eps=1e-5)


def wavlm_geometry(**over):
    g = dict(WAVLM_BASE)
    g.update(over)
    return g


def rel_position_bucket(rel: torch.Tensor, num_buckets: int = 320, max_distance: int = 800) -> torch.Tensor:
    """HF:modeling_wavlm.py:253-271 (fp32 log, truncation toward zero)."""
    nb = num_buckets // 2
    buckets = (rel > 0).to(torch.long) * nb
    rel = torch.abs(rel)
    max_exact = nb // 2
    is_small = rel < max_exact
    large = torch.log(rel.float() / max_exact)
    large = large / math.log(max_distance / max_exact)
    large = large * (nb - max_exact)
    large = (max_exact + large).to(torch.long)
    large = torch.min(large, torch.full_like(large, nb - 1))
    return buckets + torch.where(is_small, rel, large)


def wavlm_feature_extractor(sd, pre, wave, g):
    """HF:675-782 — conv0 + GroupNorm(C groups) + GELU, then conv1..6 + GELU (no bias)."""
    h = wave[:, None]
    for i, (k, s) in enumerate(zip(g["conv_kernel"], g["conv_stride"])):
        h = F.conv1d(h, sd[f"{pre}feature_extractor.conv_layers.{i}.conv.weight"], None, stride=s)
        if i == 0:
            C = h.shape[1]
            h = F.group_norm(h, C, sd[f"{pre}feature_extractor.conv_layers.0.layer_norm.weight"],
                             sd[f"{pre}feature_extractor.conv_layers.0.layer_norm.bias"], 1e-5)
        h = F.gelu(h)
    return h  # [B, C, S]


def wavlm_forward(sd: Dict[str, torch.Tensor], wave: torch.Tensor, g: dict, pre: str = "") -> torch.Tensor:
    """WavLMModel.forward (HF:1032-1088) with attention_mask=None in eval mode -> last_hidden_state."""
    eps = g["layer_norm_eps"]
    E, H = g["hidden_size"], g["num_attention_heads"]
    dh = E // H
    fe = wavlm_feature_extractor(sd, pre, wave, g).transpose(1, 2)           # HF:1055-1056
    x = F.layer_norm(fe, (fe.shape[-1],), sd[pre + "feature_projection.layer_norm.weight"],
                     sd[pre + "feature_projection.layer_norm.bias"], eps)    # HF:102
    x = F.linear(x, sd[pre + "feature_projection.projection.weight"], sd[pre + "feature_projection.projection.bias"])
    # positional conv embedding, weight_norm(dim=2) — HF:37-90
    gw = sd[pre + "encoder.pos_conv_embed.conv.parametrizations.weight.original0"]
    vw = sd[pre + "encoder.pos_conv_embed.conv.parametrizations.weight.original1"]
    w = gw * vw / vw.norm(dim=(0, 1), keepdim=True)
    kpos = g["num_conv_pos_embeddings"]
    pos = F.conv1d(x.transpose(1, 2), w, sd[pre + "encoder.pos_conv_embed.conv.bias"], padding=kpos // 2,
                   groups=g["num_conv_pos_embedding_groups"])
    if kpos % 2 == 0:
        pos = pos[:, :, :-1]
    x = x + F.gelu(pos).transpose(1, 2)                                     # HF:404-405
    x = F.layer_norm(x, (E,), sd[pre + "encoder.layer_norm.weight"], sd[pre + "encoder.layer_norm.bias"], eps)
    B, S, _ = x.shape
    rel = torch.arange(S)[None, :] - torch.arange(S)[:, None]
    bucket = rel_position_bucket(rel, g["num_buckets"], g["max_bucket_distance"])
    bias = sd[pre + "encoder.layers.0.attention.rel_attn_embed.weight"][bucket].permute(2, 0, 1)  # [H,S,S]
    for i in range(g["num_hidden_layers"]):
        lp = f"{pre}encoder.layers.{i}."
        a = lp + "attention."
        # gate from the layer input, per head (HF:166-180)
        gh = x.view(B, S, H, dh).permute(0, 2, 1, 3)
        rp = F.linear(gh, sd[a + "gru_rel_pos_linear.weight"], sd[a + "gru_rel_pos_linear.bias"])
        rp = rp.view(B, H, S, 2, 4).sum(-1)
        ga, gb = torch.sigmoid(rp).chunk(2, dim=-1)
        gate = ga * (gb * sd[a + "gru_rel_pos_const"].view(1, H, 1, 1) - 1.0) + 2.0   # [B,H,S,1]
        gbias = gate * bias[None]                                            # [B,H,S,S]
        q = F.linear(x, sd[a + "q_proj.weight"], sd[a + "q_proj.bias"]).view(B, S, H, dh).transpose(1, 2)
        k = F.linear(x, sd[a + "k_proj.weight"], sd[a + "k_proj.bias"]).view(B, S, H, dh).transpose(1, 2)
        v = F.linear(x, sd[a + "v_proj.weight"], sd[a + "v_proj.bias"]).view(B, S, H, dh).transpose(1, 2)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(dh) + gbias
        o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, S, E)
        o = F.linear(o, sd[a + "out_proj.weight"], sd[a + "out_proj.bias"])
        x = F.layer_norm(x + o, (E,), sd[lp + "layer_norm.weight"], sd[lp + "layer_norm.bias"], eps)   # HF:313-317
        ffh = F.gelu(F.linear(x, sd[lp + "feed_forward.intermediate_dense.weight"],
                              sd[lp + "feed_forward.intermediate_dense.bias"]))
        ff = F.linear(ffh, sd[lp + "feed_forward.output_dense.weight"], sd[lp + "feed_forward.output_dense.bias"])
        x = F.layer_norm(x + ff, (E,), sd[lp + "final_layer_norm.weight"], sd[lp + "final_layer_norm.bias"], eps)
    return x


def acoustic_encoder(sd, wave, g, d_model):
    """models/acoustic_encoder.py:84-128 with lengths=None: (feats, None, None)."""
    h = wavlm_forward(sd, wave, g, pre="backbone.")
    if g["hidden_size"] != d_model:
        h = F.linear(h, sd["proj.weight"], sd["proj.bias"])
    return h


# ------------------------------------------------------------------------------------------------
# Full train step — train.py:340-443 (teacher-forced t / xt), AdamW + clip_grad_norm_(5.0)
# ------------------------------------------------------------------------------------------------
class OracleAdamW:
    """torch.optim.AdamW single-tensor semantics (lr 2e-4, wd 0.01, betas .9/.999, eps 1e-8);
    parameters whose grad is None are skipped entirely (train.py:400 set_to_none)."""

    def __init__(self, lr=2e-4, wd=0.01, b1=0.9, b2=0.999, eps=1e-8):
        self.lr, self.wd, self.b1, self.b2, self.eps = lr, wd, b1, b2, eps
        self.state = {}

    def step(self, params: Dict[str, torch.Tensor], grads: Dict[str, Optional[torch.Tensor]]):
        for n, p in params.items():
            g = grads.get(n)
            if g is None:
                continue
            st = self.state.setdefault(n, {"step": 0, "m": torch.zeros_like(p), "v": torch.zeros_like(p)})
            st["step"] += 1
            p.mul_(1 - self.lr * self.wd)
            st["m"].lerp_(g, 1 - self.b1)
            st["v"].mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            bc1 = 1 - self.b1 ** st["step"]
            bc2 = 1 - self.b2 ** st["step"]
            denom = (st["v"].sqrt() / math.sqrt(bc2)).add_(self.eps)
            p.addcdiv_(st["m"], denom, value=-self.lr / bc1)


def clip_grads(grads: Dict[str, Optional[torch.Tensor]], max_norm: float = 5.0):
    gs = [g for g in grads.values() if g is not None]
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g, 2) for g in gs]), 2)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for g in gs:
        g.mul_(coef)
    return total


def oracle_train_step(params: Dict[str, torch.Tensor], enc_sd, enc_geom, wave, x0, t, xt, cfg: dict,
                      optim: OracleAdamW, global_step: int, betas, alpha_bar, c: Optional[torch.Tensor] = None,
                      dropout: float = 0.0, seed: int = 0, taps: Optional[list] = None):
    """One teacher-forced step of train_one_epoch (train.py:342-423). `params` holds the trainable
    tensors under the names decoder.*, s_proj.*, t_embed.*, t_proj.* and is updated in place.
    cfg keys: d_model, nhead, num_layers, pad_id, n_step_fd, tau, lambda_offdiag.
    Optional: `c` replaces the encoder output (the step from a given acoustic condition, e.g. the GPU's own, to
    separate the encoder's rounding from the decoder's); `dropout` / `seed` run the decoder's dropout sites under the
    RNG contract (decoder_forward); `taps` collects the block outputs (their .grad after backward).
    Returns dict(kl, lfd, loss, c, logits, dlogits, grads)."""
    d = cfg["d_model"]
    if c is None:
        with torch.no_grad():
            c = acoustic_encoder(enc_sd, wave, enc_geom, d)                 # train.py:349
    leaves = {n: p.detach().clone().requires_grad_(True) for n, p in params.items()}
    dec_sd = {n[len("decoder."):]: p for n, p in leaves.items() if n.startswith("decoder.")}
    x_mask = x0 != cfg["pad_id"]
    logits = decoder_forward(dec_sd, xt, t, c, x_mask, cfg["nhead"], cfg["num_layers"], cfg["pad_id"],
                             dropout=dropout, seed=seed, taps=taps)
    logits.retain_grad()
    B, L, V = logits.shape
    # KL (train.py:190-255) by its direct formula, differentiated by autograd
    eps = 1e-8
    xhat = torch.softmax(logits, -1)
    bt = betas[t - 1].view(B, 1, 1)
    bp = torch.where(t.eq(1), torch.zeros(()), betas[(t - 2).clamp(min=0)]).view(B, 1, 1)
    xt_oh = F.one_hot(xt, V).float()
    x0_oh = F.one_hot(x0, V).float()
    M = bt / V + (1 - bt) * xt_oh
    dq = bt[..., 0] / V + (1 - bt[..., 0]) * (x0_oh * xt_oh).sum(-1)
    dp = bt[..., 0] / V + (1 - bt[..., 0]) * torch.gather(xhat, -1, xt[..., None])[..., 0]
    Q = M * ((1 - bp) * x0_oh + bp / V) / (dq[..., None] + eps)
    P = M * ((1 - bp) * xhat + bp / V) / (dp[..., None] + eps)
    klt = (Q * (torch.log(Q + eps) - torch.log(P + eps))).sum(-1)
    valid = x_mask.float()
    kl = ((klt * valid).sum(1) / (valid.sum(1) + eps)).mean()
    loss = kl
    lfd_v = None
    if global_step % cfg["n_step_fd"] == 0:                                  # train.py:372
        z_text = F.linear(torch.softmax(logits, -1) @ leaves["t_embed.proj.weight"].T,
                          leaves["t_proj.proj.net.0.weight"], leaves["t_proj.proj.net.0.bias"])
        z_speech = F.linear(c, leaves["s_proj.proj.net.0.weight"], leaves["s_proj.proj.net.0.bias"])
        z_speech = align_speech(z_speech, L)
        w_t = alpha_bar[t - 1].mean()                                         # train.py:390
        lfd_v = lfd_loss(z_speech, z_text, cfg["lambda_offdiag"])
        loss = loss + cfg["tau"] * w_t * lfd_v
    loss.backward()
    grads = {}
    for n, p in leaves.items():
        # projector grads are None on non-L_fd steps (set_to_none semantics)
        grads[n] = p.grad.detach().clone() if p.grad is not None else None
    raw = {n: (None if g is None else g.clone()) for n, g in grads.items()}
    clip_grads(grads, 5.0)
    optim.step(params, grads)
    return dict(kl=float(kl.detach()), lfd=None if lfd_v is None else float(lfd_v.detach()), loss=float(loss.detach()), c=c,
                logits=logits.detach(), dlogits=logits.grad, grads=raw)


# ------------------------------------------------------------------------------------------------
# Jumpy sampler: sampler/jumpy_sampler.py:167-293 + q_posterior_multi_step
# fddm/sched/diffusion_scheduler.py:106-208.
# ------------------------------------------------------------------------------------------------
def jump_coeffs(betas: np.ndarray, K: int, T: int, t: int, delta: int):
    """(a_cum, b_cum, a_tg, b_tg) for one batch element, in the reference's fp32 scalar arithmetic:
    M_{t:t-Δ+1} ≈ a_cum I + b_cum 11ᵀ over s = t..t-Δ+1 (diffusion_scheduler.py:146-167) exactly as
    executed: a' = a_s·a, then b' = a_s·b + b_s(a' + K b) — `a_old` (:160) is a 0-d view of
    a_cumulative, so the store at :163 is visible to the b update at :164 (pinned by the jumpy
    fixture). M_{t-Δ} = a_tg I + b_tg 11ᵀ, identity at t-Δ = 0 (:170-185)."""
    f = np.float32
    betas = np.asarray(betas, dtype=np.float32)
    a, b = f(1.0), f(0.0)
    for s in range(t, t - delta, -1):
        if 1 <= s <= T:
            bs = betas[s - 1]
            a_s = f(1.0) - bs
            b_s = bs / f(K)
            a = a_s * a
            b = a_s * b + b_s * (a + f(K) * b)
    tg = t - delta
    if tg > 0 and tg <= T:
        a_tg, b_tg = f(1.0) - betas[tg - 1], betas[tg - 1] / f(K)
    else:
        a_tg, b_tg = f(1.0), f(0.0)
    return a, b, a_tg, b_tg


def jump_argmax(logits: torch.Tensor, xt: torch.Tensor, t: torch.Tensor, delta: int, betas, K: int, T: int):
    """argmax_k q(x_{t-Δ}=k | x_t, x̂0=softmax(logits)) (diffusion_scheduler.py:187-206 + argmax,
    jumpy_sampler.py:212-215) in closed form. With x_t one-hot, the unnormalised posterior is
    (a_cum[k=x_t] + b_cum)(a_tg x̂_k + b_tg Σx̂): every k ≠ x_t shares the factor b_cum, so the winner
    is x_t or o = first argmax_{k≠x_t} x̂_k. Returns (next indices, margin) where margin is the
    relative score gap (near-ties, |margin| ~ fp32 eps, may round either way in the reference)."""
    B, L, V = logits.shape
    delta = min(int(delta), int(t.min()))
    z = logits.double()
    p = torch.softmax(z, -1)
    out = torch.empty(B, L, dtype=torch.long)
    margin = torch.empty(B, L, dtype=torch.float64)
    for bi in range(B):
        a, b, a_tg, b_tg = (float(v) for v in jump_coeffs(betas, K, T, int(t[bi]), delta))
        for li in range(L):
            x = int(xt[bi, li])
            row = p[bi, li].clone()
            px = float(row[x])
            row[x] = -1.0
            o = int(torch.argmax(row))
            so = b * (a_tg * float(row[o]) + b_tg)
            sx = (a + b) * (a_tg * px + b_tg)
            if sx > so or (sx == so and x < o):
                out[bi, li] = x
            else:
                out[bi, li] = o
            margin[bi, li] = (sx - so) / max(sx, so)
    return out, margin


def alpha_bar_at_t_train(alpha_bar, t_infer: int, T_infer: int, T_train: int):
    """jumpy_sampler.py:217-233 (fast mode): nearest training step of t_infer; ᾱ₀ = 1. Indexes the
    0-based alpha_bar[T] with a 1..T_train step exactly as the reference does (IndexError at T_train)."""
    if t_infer <= 0:
        return np.float32(1.0)
    tf = max(1.0, min(float(T_train), float(t_infer) / float(max(1, T_infer)) * float(T_train)))
    return np.float32(np.asarray(alpha_bar, dtype=np.float32)[int(round(tf))])


def jumpy_sample(logits_fn, xT: torch.Tensor, T_infer: int, r: int, betas, alpha_bar, K: int, T_train: int,
                 mode: str = "exact"):
    """DiffusionJumpySampler.sample with greedy decoding (jumpy_sampler.py:235-293): from x_T jump by
    Δ = min(r, t) until t = 0; returns the per-jump x_{t-Δ} and x̂0 argmaxes and the final
    x0 = argmax p_x0_last. `logits_fn(x, t_vec)` is the decoder forward."""
    B, L = xT.shape
    x, t = xT.clone(), T_infer
    xs, x0hats, logits = [], [], None
    while t > 0:
        delta = min(r, t)
        tv = torch.full((B,), t, dtype=torch.long)
        logits = logits_fn(x, tv)
        if mode == "exact":
            nx, _ = jump_argmax(logits, x, tv, delta, betas, K, T_train)
        else:
            ab = float(alpha_bar_at_t_train(alpha_bar, max(0, t - delta), T_infer, T_train))
            p = torch.softmax(logits.double(), -1)
            nx = (ab * p + (1.0 - ab) / K).argmax(-1)
        xs.append(nx)
        x0hats.append(logits.argmax(-1))
        x = nx
        t -= delta
    return torch.stack(xs), torch.stack(x0hats), logits.argmax(-1)
