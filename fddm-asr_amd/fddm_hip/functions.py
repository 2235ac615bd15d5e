"""torch.autograd.Functions of the train step. Each forward/backward is a fixed sequence of
libfddm_hip launches on the current stream; activations are saved in the compute dtype (bf16 / f32)
with the residual stream, LayerNorm statistics and softmax log-sum-exps in fp32.
"""
from __future__ import annotations

import math
import weakref

import torch
import torch.nn.functional as F

from . import ops, runtime as rt

F32 = torch.float32


def _t(x):
    """compute-dtype view/copy of an activation"""
    cd = rt.compute_dtype()
    return x if x.dtype == cd else ops.cast(x.contiguous(), cd)


def _gdst(p, zero=False):
    """(destination, in_arena) for p's gradient: its GradArena view, accumulated in place by the kernels
    (the Function then returns None for p), or a fresh fp32 tensor returned to autograd."""
    s = rt.grad_slot(p)
    if s is not None:
        return s, True
    return (torch.zeros if zero else torch.empty)(p.shape, device=p.device, dtype=F32), False


def _ret(t, in_arena):
    return None if in_arena else t


def _dw_flush(jobs):
    """Run deferred weight-gradient GEMMs (dy, x, dW, db), all accumulating into zeroed or arena buffers:
    one grouped launch in bf16, one GEMM per job otherwise (fp32 parity mode)."""
    if jobs and all(j[0].dtype == torch.bfloat16 and j[1].dtype == torch.bfloat16 for j in jobs):
        ops.linear_dw_grouped(jobs)
    else:
        for dy, x, dW, db in jobs:
            ops.linear_dw(dy, x, out=dW, accumulate=True, db=db)


# ------------------------------------------------------------------------------- generic Linear
class LinearFn(torch.autograd.Function):
    """y = x W^T + b (f32 out) — SpeechProjector / TextProjector / encoder proj (models/projection.py)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        shp = x.shape
        x2 = _t(x.reshape(-1, shp[-1]).contiguous())
        w = rt.wt(weight)
        y = ops.linear(x2, w, bias, out_dtype=F32)
        ctx.save_for_backward(x2, weight, bias)
        ctx.shp = shp
        return y.view(*shp[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight, bias = ctx.saved_tensors
        dy2 = dy.reshape(-1, weight.shape[0]).contiguous()
        dyt = _t(dy2)
        dx = dW = db = None
        aw = ab = False
        if ctx.needs_input_grad[0]:
            dx = ops.linear_dx(dyt, rt.wt(weight)).view(ctx.shp)
        if bias is not None and ctx.needs_input_grad[2]:
            db, ab = _gdst(bias)
        if ctx.needs_input_grad[1]:
            dW, aw = _gdst(weight)
            if db is not None and ab != aw:      # bias and weight disagree on accumulation: separate sum
                ops.linear_dw(dyt, x2, out=dW, accumulate=aw)
                ops.colsum(dy2, out=db, accumulate=ab)
            else:
                ops.linear_dw(dyt, x2, out=dW, accumulate=aw, db=db)
        elif db is not None:
            ops.colsum(dy2, out=db, accumulate=ab)
        return dx, _ret(dW, aw), _ret(db, ab)


def linear(x, weight, bias=None):
    return LinearFn.apply(x, weight, bias)


# ------------------------------------------------------------------------------ token embedding
class EmbedFn(torch.autograd.Function):
    """x = tok_emb[xt] + t_bias[b]   (models/denoise_decoder.py:254, 274). Returns (x f32, x_T)."""

    @staticmethod
    def forward(ctx, xt, E, tbias, pad_id):
        B, L = xt.shape
        d = E.shape[1]
        x = torch.empty(B * L, d, device=E.device, dtype=F32)
        cd = rt.compute_dtype()
        xT = torch.empty(B * L, d, device=E.device, dtype=cd)
        ops.embed_fwd(xt.contiguous(), E.detach(), tbias.detach().contiguous(), x, xT, L)
        ctx.set_materialize_grads(False)     # xT is non-differentiable: no zero-filled gradient for it
        ctx.save_for_backward(xt)
        ctx.E = (E,)
        ctx.pad_id, ctx.L, ctx.V = pad_id, L, E.shape[0]
        ctx.mark_non_differentiable(xT)
        return x, xT

    @staticmethod
    def backward(ctx, dx, _dxT):
        (xt,) = ctx.saved_tensors
        d = dx.shape[1]
        B = xt.shape[0]
        E, = ctx.E
        dE, aE = _gdst(E, zero=True)
        dtb = torch.zeros(B, d, device=dx.device, dtype=F32)
        ops.embed_bwd(xt.contiguous(), dx.contiguous(), dE, dtb, ctx.L, ctx.pad_id)
        return None, _ret(dE, aE), dtb, None


# ------------------------------------------------------------------------- decoder conditioning
def sinusoid(t, d, max_steps):
    """SinusoidalTimeEmbedding's feature map (models/denoise_decoder.py:92-119), on the device (fddm_time_embed)."""
    if t.dim() == 0:
        t = t[None]
    return ops.time_embed(t.to(torch.int64).contiguous(), d, max_steps)


class CondFn(torch.autograd.Function):
    """The decoder's conditioning path as one Function: t_bias = time_proj(mlp(sinusoid(t)))
    (models/denoise_decoder.py:92-119, 272-274) and the FiLM projections scale_l / shift_l = pooled W^T + b of
    every block (:74-89; pooled = time-mean of the acoustic condition, no grad). All of it runs on the small
    row-batch fp32 kernels (csrc/small.hip): forward = time embedding + 3 Linears (SiLU fused) + ONE launch for all
    2*NL FiLM projections; backward = the two input-gradient Linears (SiLU' fused) and the weight / bias gradients
    of all of them in one launch, straight into the parameters' gradient slots. `gbuf` [2*NL, B, d] (zeroed by the
    caller) is where the blocks' LayerNorm backward accumulates dFiLM."""

    @staticmethod
    def forward(ctx, t, pooled, gbuf, d, max_steps, *params):
        W1, b1, W2, b2, Wp, bp = params[:6]
        film = params[6:]
        nf = len(film) // 2
        with torch.no_grad():
            emb = sinusoid(t, d, max_steps)                                      # [B, d]
            Bt = emb.shape[0]
            dev = emb.device
            pre = torch.empty(Bt, W1.shape[0], device=dev, dtype=F32)
            h = torch.empty_like(pre)
            ops.small_linear(emb, [W1.detach()], [b1.detach()], [pre], [h], act=1)
            te = torch.empty(Bt, W2.shape[0], device=dev, dtype=F32)
            ops.small_linear(h, [W2.detach()], [b2.detach()], [te])
            tb = torch.empty(Bt, Wp.shape[0], device=dev, dtype=F32)
            ops.small_linear(te, [Wp.detach()], [bp.detach()], [tb])
            B = pooled.shape[0]
            f12 = torch.empty(nf, B, d, device=dev, dtype=F32)
            if nf:
                ops.small_linear(pooled.contiguous(), [w.detach() for w in film[0::2]], [b.detach() for b in film[1::2]],
                                 [f12[i] for i in range(nf)])
        ctx.save_for_backward(emb, pre, h, te, pooled, gbuf, *params)
        ctx.nf = nf
        return (tb,) + tuple(f12[i] for i in range(nf))

    @staticmethod
    def backward(ctx, dtb, *dfilm):
        emb, pre, h, te, pooled, gbuf, *params = ctx.saved_tensors
        W1, b1, W2, b2, Wp, bp = params[:6]
        film = params[6:]
        nf = ctx.nf
        B, d = pooled.shape
        dev = pooled.device
        grads = [None] * len(params)
        # FiLM: the blocks accumulated into gbuf and handed back its slices; anything else is stacked
        if all(g is not None and g.data_ptr() == gbuf[i].data_ptr() for i, g in enumerate(dfilm)):
            dfl = gbuf
        else:
            dfl = torch.stack([g if g is not None else torch.zeros(B, d, device=dev) for g in dfilm])
        G = [_gdst(p_, zero=True) for p_ in film]
        jobs = [(dfl[i], pooled, G[2 * i][0], G[2 * i + 1][0]) for i in range(nf)]
        T = None
        if dtb is not None:
            dtb = dtb.contiguous()
            T = [_gdst(p_, zero=True) for p_ in (W1, b1, W2, b2, Wp, bp)]
            jobs.append((dtb, te, T[4][0], T[5][0]))
        ops.small_dw(jobs)                                        # FiLM + time_proj weight / bias gradients
        for i in range(2 * nf):
            grads[6 + i] = _ret(*G[i])
        if dtb is not None:
            # tb = te Wp^T + bp, te = h W2^T + b2, h = silu(pre), pre = emb W1^T + b1
            Bt = dtb.shape[0]
            dte = torch.empty(Bt, Wp.shape[1], device=dev, dtype=F32)
            ops.small_linear(dtb, [Wp.detach()], None, [dte], transpose_w=True)
            dpre = torch.empty(Bt, W2.shape[1], device=dev, dtype=F32)
            ops.small_linear(dte, [W2.detach()], None, [dpre], act=2, aux=pre, transpose_w=True)
            ops.small_dw([(dte, h, T[2][0], T[3][0]), (dpre, emb, T[0][0], T[1][0])])
            for i in range(6):
                grads[i] = _ret(*T[i])
        return (None, None, None, None, None) + tuple(grads)


# -------------------------------------------------------------------------------- decoder block
def _film_split(fs):
    return fs.contiguous()


class DecoderBlockFn(torch.autograd.Function):
    """DecoderBlock.forward (models/denoise_decoder.py:147-192) as one fused sequence:
    RoPE -> self-attn (kpm, dropout) -> +drop -> LN1 -> cross-attn -> +drop -> LN2 -> FiLM ->
    FF(GELU, dropout) -> +drop -> LN3.  Inputs: x (f32 [N,d], differentiable), xT (compute dtype copy),
    cT (cond, compute dtype [B*S,d], no grad), key_keep (u8 [B,L]), film scale/shift [B,d] (diff.),
    then the 18 block parameters. Dropout sites use rng streams 6*layer + {1..6}."""

    @staticmethod
    def forward(ctx, x, xT, cT, key_keep, fscale, fshift, meta, *params):
        (sa_w, sa_b, so_w, so_b, ca_w, ca_b, co_w, co_b, f0_w, f0_b, f3_w, f3_b,
         n1w, n1b, n2w, n2b, n3w, n3b) = params
        B, L, S, H, layer, p, seed, cos, sin = meta[:9]
        N, d = x.shape
        dev = x.device
        cd = rt.compute_dtype()
        st = 6 * layer
        W = {k: rt.wt(v) for k, v in (("sa", sa_w), ("so", so_w), ("ca", ca_w), ("co", co_w), ("f0", f0_w),
                                       ("f3", f3_w))}
        # 1. RoPE on the block input (q = k = rope(x), v = x): written by the previous block's LN3 when it was
        # given a hand-off (meta[12]), else here
        xr = meta[12] if len(meta) > 12 else None
        if xr is None:
            xr = torch.empty(N, d, device=dev, dtype=cd)
            ops.rope_fwd(x, cos, sin, xr, L)
        handoff = meta[13] if len(meta) > 13 else None
        qk = ops.linear(xr, W["sa"][: 2 * d], sa_b[: 2 * d], out_dtype=cd)
        v = ops.linear(xT, W["sa"][2 * d:], sa_b[2 * d:], out_dtype=cd)
        o = torch.empty(N, d, device=dev, dtype=cd)
        lse = torch.empty(B * H, L, device=dev, dtype=F32)
        # dropout keep bits of both attention sites: written for every block ahead of the forward
        # (DenoisingTransformerDecoder._drop_bits, two launches per step) or here by the forward itself
        pre = meta[11] if len(meta) > 11 else None
        ready = pre is not None and p > 0
        bits_s = pre[0] if ready else (ops.drop_bits(B, H, L, L, dev) if p > 0 else None)
        bits_c = pre[1] if ready else (ops.drop_bits(B, H, L, S, dev) if p > 0 else None)
        fwd_s = lambda: ops.attn_fwd(qk, qk[:, d:], v, o, lse, B, H, L, L, key_keep=key_keep, drop_p=p,  # noqa: E731
                                     seed=seed, rng_stream=st + 1, dbits=bits_s, bits_ready=ready)
        with rt.probe("decoder.self_attn_fwd", replay=fwd_s):
            fwd_s()
        y = ops.linear(o, W["so"], so_b, out_dtype=cd)
        s1 = torch.empty(N, d, device=dev, dtype=F32)
        m1 = torch.empty(N, device=dev, dtype=F32)
        r1 = torch.empty(N, device=dev, dtype=F32)
        x1 = torch.empty(N, d, device=dev, dtype=F32)
        x1T = torch.empty(N, d, device=dev, dtype=cd) if cd != F32 else x1
        ops.ln_fwd(x, y, n1w, n1b, out_f32=x1, out_t=x1T if cd != F32 else None, save_s=s1, mean=m1, rstd=r1,
                   drop_p=p, seed=seed, rng_stream=st + 2)
        # 2. cross-attention to the acoustic condition
        qc = ops.linear(x1T, W["ca"][:d], ca_b[:d], out_dtype=cd)
        kvc = meta[10] if len(meta) > 10 and meta[10] is not None else \
            ops.linear(cT, W["ca"][d:], ca_b[d:], out_dtype=cd)      # (precomputed for all blocks in one GEMM)
        oc = torch.empty(N, d, device=dev, dtype=cd)
        lsec = torch.empty(B * H, L, device=dev, dtype=F32)
        fwd_c = lambda: ops.attn_fwd(qc, kvc, kvc[:, d:], oc, lsec, B, H, L, S, drop_p=p, seed=seed,  # noqa: E731
                                     rng_stream=st + 3, dbits=bits_c, bits_ready=ready)
        with rt.probe("decoder.cross_attn_fwd", replay=fwd_c):
            fwd_c()
        yc = ops.linear(oc, W["co"], co_b, out_dtype=cd)
        s2 = torch.empty(N, d, device=dev, dtype=F32)
        m2 = torch.empty(N, device=dev, dtype=F32)
        r2 = torch.empty(N, device=dev, dtype=F32)
        x2 = torch.empty(N, d, device=dev, dtype=F32)
        x2T = torch.empty(N, d, device=dev, dtype=cd) if cd != F32 else x2
        fsc, fsh = fscale.detach().contiguous(), fshift.detach().contiguous()
        ops.ln_fwd(x1, yc, n2w, n2b, out_f32=x2, out_t=x2T if cd != F32 else None, save_s=s2, mean=m2, rstd=r2,
                   film=(fsc, fsh), rows_per_batch=L, drop_p=p, seed=seed, rng_stream=st + 4)
        # 3. feed-forward
        FF = f0_w.shape[0]
        hpre = torch.empty(N, FF, device=dev, dtype=cd)
        hact = torch.empty(N, FF, device=dev, dtype=cd)
        ops.linear(x2T, W["f0"], f0_b, out=hpre, epi=ops.EPI_GELU, C2=hact, drop_p=p, seed=seed, rng_stream=st + 5)
        y3 = ops.linear(hact, W["f3"], f3_b, out_dtype=cd)
        s3 = torch.empty(N, d, device=dev, dtype=F32)
        m3 = torch.empty(N, device=dev, dtype=F32)
        r3 = torch.empty(N, device=dev, dtype=F32)
        x3 = torch.empty(N, d, device=dev, dtype=F32)
        x3T = torch.empty(N, d, device=dev, dtype=cd)
        rope = None
        # the next block's rope(x) from the same pass, where the fused LN kernel takes the shape (fddm_ln_fwd: bf16,
        # d % 16 == 0, d <= 1024); otherwise handoff stays empty and the next block runs its own rope_fwd
        if handoff is not None and cd == torch.bfloat16 and d % 16 == 0 and d <= 1024:
            handoff["xr"] = torch.empty(N, d, device=dev, dtype=cd)
            rope = (cos, sin, handoff["xr"], L)
        ops.ln_fwd(x2, y3, n3w, n3b, out_f32=x3, out_t=x3T, save_s=s3, mean=m3, rstd=r3,
                   drop_p=p, seed=seed, rng_stream=st + 6, rope=rope)
        ctx.save_for_backward(xT, xr, qk, v, o, lse, s1, m1, r1, x1T, qc, kvc, oc, lsec, s2, m2, r2, x2T, hpre, hact,
                              s3, m3, r3, cT, key_keep, fsc, *params)
        ctx.meta = meta
        ctx.bits = (bits_s, bits_c)
        ctx.mark_non_differentiable(x3T)
        ctx.set_materialize_grads(False)     # x3T's gradient is never used: no zero fill per block
        return x3, x3T

    @staticmethod
    def backward(ctx, dx3, _dx3T):
        (xT, xr, qk, v, o, lse, s1, m1, r1, x1T, qc, kvc, oc, lsec, s2, m2, r2, x2T, hpre, hact, s3, m3, r3, cT,
         key_keep, fsc, *params) = ctx.saved_tensors
        (sa_w, sa_b, so_w, so_b, ca_w, ca_b, co_w, co_b, f0_w, f0_b, f3_w, f3_b,
         n1w, n1b, n2w, n2b, n3w, n3b) = params
        B, L, S, H, layer, p, seed, cos, sin = ctx.meta[:9]
        gfilm = ctx.meta[9] if len(ctx.meta) > 9 else None
        st = 6 * layer
        N, d = dx3.shape
        dev = dx3.device
        cd = rt.compute_dtype()
        W = {k: rt.wt(v_) for k, v_ in (("sa", sa_w), ("so", so_w), ("ca", ca_w), ("co", co_w), ("f0", f0_w),
                                         ("f3", f3_w))}
        # gradient destinations: arena views (accumulated in place) or fresh tensors
        # (every destination accumulates: the weight gradients are deferred to one grouped launch at the end)
        G = [_gdst(p_, zero=True) for p_ in params]
        (gsa_w, asa), (gsa_b, _), (gso_w, aso), (gso_b, _), (gca_w, aca), (gca_b, _), (gco_w, aco), (gco_b, _), \
            (gf0_w, af0), (gf0_b, _), (gf3_w, af3), (gf3_b, _), (gn1w, _), (gn1b, _), (gn2w, _), (gn2b, _), \
            (gn3w, _), (gn3b, _) = G
        dx3 = dx3.contiguous()
        # the three LayerNorms' dgamma / dbeta slab sums, added in one fold launch before the weight gradients
        lnp = ops.LnPartials()
        # LN3
        dx2 = torch.empty(N, d, device=dev, dtype=F32)
        dy3 = torch.empty(N, d, device=dev, dtype=cd)
        ops.ln_bwd(dx3, s3, m3, r3, n3w, n3b, dres=dx2, dy_t=dy3, dgamma=gn3w, dbeta=gn3b, drop_p=p,
                   seed=seed, rng_stream=st + 6, partials=lnp)
        # FF
        dw_jobs = [(dy3, hact, gf3_w, gf3_b)]
        FF = f0_w.shape[0]
        dh = torch.empty(N, FF, device=dev, dtype=cd)
        ops.linear_dx(dy3, W["f3"], out=dh, epi=ops.EPI_DGELU, C2=hpre, drop_p=p, seed=seed, rng_stream=st + 5)
        dw_jobs.append((dh, x2T, gf0_w, gf0_b))
        ops.linear_dx(dh, W["f0"], out=dx2, accumulate=True)
        # LN2 + FiLM
        dx1 = torch.empty(N, d, device=dev, dtype=F32)
        dyc = torch.empty(N, d, device=dev, dtype=cd)
        if gfilm is not None:   # zeroed slices of CondFn's FiLM-gradient buffer (one fill per step)
            dfs, dfh = gfilm
        else:
            dfs = torch.zeros(B, d, device=dev, dtype=F32)
            dfh = torch.zeros(B, d, device=dev, dtype=F32)
        ops.ln_bwd(dx2, s2, m2, r2, n2w, n2b, dres=dx1, dy_t=dyc, dgamma=gn2w, dbeta=gn2b, film_scale=fsc,
                   dfilm=(dfs, dfh), rows_per_batch=L, drop_p=p, seed=seed, rng_stream=st + 4, partials=lnp)
        # cross out-proj + attention
        dw_jobs.append((dyc, oc, gco_w, gco_b))
        doc = ops.linear_dx(dyc, W["co"], out_dtype=cd)
        dqc = torch.empty(N, d, device=dev, dtype=cd)
        dkvc = torch.empty(B * S, 2 * d, device=dev, dtype=cd)
        bits_s, bits_c = ctx.bits
        bwd_c = lambda: ops.attn_bwd(qc, kvc, kvc[:, d:], oc, doc, lsec, dqc, dkvc, dkvc[:, d:], B, H, L, S,  # noqa: E731
                                     drop_p=p, seed=seed, rng_stream=st + 3, dbits=bits_c)
        with rt.probe("decoder.cross_attn_bwd", replay=bwd_c):
            bwd_c()
        dw_jobs += [(dqc, x1T, gca_w[:d], gca_b[:d]), (dkvc, cT, gca_w[d:], gca_b[d:])]
        ops.linear_dx(dqc, W["ca"][:d], out=dx1, accumulate=True)
        # LN1
        dx = torch.empty(N, d, device=dev, dtype=F32)
        dy = torch.empty(N, d, device=dev, dtype=cd)
        ops.ln_bwd(dx1, s1, m1, r1, n1w, n1b, dres=dx, dy_t=dy, dgamma=gn1w, dbeta=gn1b, drop_p=p, seed=seed,
                   rng_stream=st + 2, partials=lnp)
        # self out-proj + attention
        dw_jobs.append((dy, o, gso_w, gso_b))
        do = ops.linear_dx(dy, W["so"], out_dtype=cd)
        dqk = torch.empty(N, 2 * d, device=dev, dtype=cd)
        dv = torch.empty(N, d, device=dev, dtype=cd)
        bwd_s = lambda: ops.attn_bwd(qk, qk[:, d:], v, o, do, lse, dqk, dqk[:, d:], dv, B, H, L, L,  # noqa: E731
                                     key_keep=key_keep, drop_p=p, seed=seed, rng_stream=st + 1, dbits=bits_s)
        with rt.probe("decoder.self_attn_bwd", replay=bwd_s):
            bwd_s()
        dw_jobs += [(dqk, xr, gsa_w[: 2 * d], gsa_b[: 2 * d]), (dv, xT, gsa_w[2 * d:], gsa_b[2 * d:])]
        ops.linear_dx(dv, W["sa"][2 * d:], out=dx, accumulate=True)
        if not ops.linear_dx_rope(dqk, W["sa"][: 2 * d], dx, cos, sin, L):     # dx += rope_bwd(dqk W_qk)
            dxr = ops.linear_dx(dqk, W["sa"][: 2 * d])
            ops.rope_bwd(dxr, cos, sin, dx, L)
        lnp.fold()
        _dw_flush(dw_jobs)
        rt.grads_ready(params)
        grads = tuple(_ret(t_, a_) for t_, a_ in G)
        return (dx, None, None, None, dfs, dfh, None) + grads


# --------------------------------------------------------------------------------------- head
# bf16 mode: the logits gradient reaches the head backward in bf16 straight from the kernels that produce it, not
# as fp32 [B*L, V] tensors that autograd sums and a cast pass converts. The hand-over is keyed by the address of a
# live HeadFn output: KLFn leaves its gradient (computed in its forward, unscaled) in _kl_dz; on L_fd steps
# TextEmbedFn.backward (which autograd runs first) writes softmax-backward + that KL part into one bf16 buffer
# (_dlogits_bf16, flagged in _combined) and KLFn.backward then only applies its upstream scalar to its share (a
# no-op when it is 1); without L_fd, KLFn.backward scales its own buffer and hands it over. Both return no
# gradient to autograd, so HeadFn.backward (materialize_grads off) receives None and takes the buffer.
_head_outputs: dict = {}     # data_ptr -> weakref to a HeadFn output (bf16 mode)
_dlogits_bf16: dict = {}     # data_ptr -> bf16 logits gradient for HeadFn.backward
_kl_dz: dict = {}            # data_ptr -> the KL's unscaled bf16 gradient (between KLFn forward and backward)
_combined: set = set()       # data_ptrs whose _dlogits_bf16 buffer already holds text part + unscaled KL part


def _drop_handover(ptr):
    _head_outputs.pop(ptr, None)
    _dlogits_bf16.pop(ptr, None)
    _kl_dz.pop(ptr, None)
    _combined.discard(ptr)


class HeadFn(torch.autograd.Function):
    """logits = h W^T + b in fp32 (models/denoise_decoder.py:286)."""

    @staticmethod
    def forward(ctx, x, xT, weight, bias):
        w = rt.wt(weight)
        logits = ops.linear(xT, w, bias, out_dtype=F32)
        ctx.save_for_backward(xT, weight)
        ctx.bias = (bias,)
        ctx.out_ptr = logits.data_ptr()
        ctx.set_materialize_grads(False)
        if xT.dtype == torch.bfloat16:
            for k in [k for k, r in _head_outputs.items() if r() is None]:   # outputs freed without a backward
                _drop_handover(k)
            _drop_handover(ctx.out_ptr)
            _head_outputs[ctx.out_ptr] = weakref.ref(logits)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        xT, weight = ctx.saved_tensors
        dz16 = _dlogits_bf16.get(ctx.out_ptr)
        _drop_handover(ctx.out_ptr)
        if dz16 is not None and (dlogits is None or all(st == 0 for st in dlogits.stride())):
            dl = dz16                                     # the handed-over gradient, already bf16
        elif dz16 is not None:
            dl = (dlogits + dz16.view(dlogits.shape)).to(torch.bfloat16).contiguous()  # + another consumer's part
        elif dlogits is None:
            dl = torch.zeros(xT.shape[0], weight.shape[0], device=xT.device, dtype=xT.dtype)
        else:
            dl = dlogits.contiguous()
            if xT.dtype == torch.bfloat16 and dl.dtype == F32:
                # one cast pass, then both head GEMMs take the bf16 LDS-DMA paths (dx: K = vocab, dW: K = tokens)
                dl = ops.cast(dl, torch.bfloat16)
        w = rt.wt(weight)
        dx = ops.linear_dx(dl, w)
        dW, aw = _gdst(weight)
        db, ab = _gdst(ctx.bias[0])
        if aw != ab:
            raise RuntimeError("head weight and bias must share the grad arena")
        ops.linear_dw(dl, xT, out=dW, accumulate=aw, db=db)
        rt.grads_ready((weight, ctx.bias[0]))
        return dx, None, _ret(dW, aw), _ret(db, ab)


# -------------------------------------------------------------------------------------- KL term
class KLFn(torch.autograd.Function):
    """SchedulerAdapter.kl_term (train.py:190-255): fused closed-form KL. With a gradient wanted, ONE pass over the
    logits produces the per-token KL and its logits gradient (times the masked-mean weights); backward only applies
    the upstream scalar on the device (ops.scale_if / axpy_if_bf16: nothing to do when it is 1, the train step's
    case). bf16 mode hands the gradient to the HeadFn that produced the logits (see the module notes above)."""

    @staticmethod
    def forward(ctx, logits, xt, x0, t, mask_u8, betas):
        """mask_u8: x_mask as uint8 [B*L] (or None: plain mean over L, train.py:253)."""
        B, L, V = logits.shape
        l2 = logits.reshape(B * L, V)
        xf, x0f, tc = xt.reshape(-1).contiguous(), x0.reshape(-1).contiguous(), t.contiguous()
        ctx.shape = (B, L, V)
        ctx.handover = None
        if not ctx.needs_input_grad[0]:
            kl_tok = ops.kl_fwd(l2, xf, x0f, tc, betas, L)
            loss, _ = ops.kl_reduce(kl_tok, mask_u8, B, L, want_w=False)
            return loss
        ptr = l2.data_ptr()
        ref = _head_outputs.get(ptr)
        owner = ref() if ref is not None else None
        bf = owner is not None and owner.data_ptr() == ptr and ptr not in _dlogits_bf16 and ptr not in _kl_dz
        l2 = l2.contiguous()
        odt = torch.bfloat16 if bf else F32
        if V % 4 == 0 and V <= ops.KL_FUSED_MAX_V and l2.data_ptr() % 16 == 0:
            kl_tok, dz = ops.kl_fused(l2, xf, x0f, tc, betas, mask_u8, L, out_dtype=odt)
            loss, _ = ops.kl_reduce(kl_tok, mask_u8, B, L, want_w=False)
        else:
            # vocabularies the one-pass kernel is not built for (V % 4 != 0, V > 32768, unaligned rows): the
            # two-pass form — per-token KL, the masked-mean weights, then the weighted gradient
            kl_tok = ops.kl_fwd(l2, xf, x0f, tc, betas, L)
            loss, w = ops.kl_reduce(kl_tok, mask_u8, B, L, want_w=True)
            one = torch.ones(1, device=l2.device, dtype=F32)
            dz = ops.kl_bwd(l2, xf, x0f, tc, betas, w, one, L, out_dtype=odt)
        ctx.dz = dz
        if bf:
            ctx.handover = ptr
            _kl_dz[ptr] = dz
        return loss

    @staticmethod
    def backward(ctx, g):
        B, L, V = ctx.shape
        dz, ctx.dz = ctx.dz, None
        gs = g.reshape(1).to(F32).contiguous()
        ptr = ctx.handover
        if ptr is not None and _kl_dz.pop(ptr, None) is not None:
            if ptr in _combined:                          # the text part already added our unscaled share
                ops.axpy_if_bf16(_dlogits_bf16[ptr], dz, gs)
                return None, None, None, None, None, None
            ref = _head_outputs.get(ptr)
            if ref is not None and ref() is not None and ptr not in _dlogits_bf16:
                _dlogits_bf16[ptr] = ops.scale_if(dz, gs)
                return None, None, None, None, None, None
        ops.scale_if(dz, gs)
        return dz.float().view(B, L, V), None, None, None, None, None


# ------------------------------------------------------------------------------- TextEmbedding
class TextEmbedFn(torch.autograd.Function):
    """softmax(logits) @ W^T (models/projection.py:41-47), K = vocab."""

    @staticmethod
    def forward(ctx, logits, weight):
        shp = logits.shape
        V = shp[-1]
        l2 = logits.reshape(-1, V).contiguous()
        cd = rt.compute_dtype()
        xhat = ops.softmax_rows(l2, cd)
        z = ops.linear(xhat, rt.wt(weight), None, out_dtype=F32)
        ctx.save_for_backward(xhat, weight)
        ctx.shp = shp
        ctx.lptr = l2.data_ptr()
        return z.view(*shp[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dz):
        xhat, weight = ctx.saved_tensors
        dz2 = dz.reshape(-1, weight.shape[0]).contiguous()
        cd = rt.compute_dtype()
        dzt = _t(dz2)       # compute-dtype operand: the f32-A form fell back to the register-staged GEMM (121 us)
        dxhat = ops.linear_dx(dzt, rt.wt(weight), out_dtype=cd)
        dW, aw = _gdst(weight)           # the optimizer's aux-arena view (accumulated in place) or a fresh tensor
        ops.linear_dw(dzt, xhat, out=dW, accumulate=aw)
        dW = _ret(dW, aw)
        ptr = ctx.lptr
        kl = _kl_dz.get(ptr)
        if (kl is not None and cd == torch.bfloat16 and ptr in _head_outputs and ptr not in _dlogits_bf16
                and ptr not in _combined and xhat.shape[-1] % 8 == 0):     # fddm_softmax_bwd_add_bf16: V % 8 == 0
            # bf16 hand-over: softmax backward + the KL's (unscaled) share in one bf16 buffer for HeadFn
            _dlogits_bf16[ptr] = ops.softmax_bwd_add_bf16(xhat, dxhat, kl)
            _combined.add(ptr)
            return None, dW
        dlogits = ops.softmax_bwd_rows(xhat, dxhat)
        return dlogits.view(ctx.shp), dW


# ---------------------------------------------------------------------------------------- L_fd
class LfdFn(torch.autograd.Function):
    """lfd_loss (losses/fddm_losses.py:29-58): batch-dim standardisation + C = za~^T zb~ /(B T).

    `group` (a torch.distributed process group, or None): data-parallel form with the statistics of the GLOBAL
    batch — the column sums of the standardisation (two passes), the [D, D] cross-correlation and,
    in backward, the two column sums of the standardisation gradient are all-reduced (~1 MB per L_fd step at C2),
    so every rank gets the loss of the whole batch; each rank's input gradient is that of the global loss w.r.t.
    its own rows, scaled by the world size so the DP gradient average (sum / W) yields the global-batch gradient."""

    @staticmethod
    def forward(ctx, z_a, z_b, lam, eps, group=None):
        B, T, D = z_a.shape
        cd = rt.compute_dtype()
        a2 = z_a.reshape(B, T * D).float().contiguous()
        b2 = z_b.reshape(B, T * D).float().contiguous()
        if group is None:
            za, isa = ops.lfd_std_fwd(a2, cd, eps)
            zb, isb = ops.lfd_std_fwd(b2, cd, eps)
            N, W = B, 1
        else:
            import torch.distributed as dist
            W = dist.get_world_size(group)
            N = B * W          # every rank holds B rows (the DP contract the KL average already relies on)
            C = T * D
            st = torch.empty(2 * C, device=z_a.device, dtype=F32)
            ops.lfd_colstat(a2, st[:C])
            ops.lfd_colstat(b2, st[C:])
            dist.all_reduce(st, group=group)
            sq = torch.empty(2 * C, device=z_a.device, dtype=F32)
            ops.lfd_colstat(a2, sq[:C], st[:C], 1.0 / N)
            ops.lfd_colstat(b2, sq[C:], st[C:], 1.0 / N)
            dist.all_reduce(sq, group=group)
            za, isa = ops.lfd_std_apply(a2, cd, st[:C], sq[:C], 1.0 / N, eps)
            zb, isb = ops.lfd_std_apply(b2, cd, st[C:], sq[C:], 1.0 / N, eps)
        za2, zb2 = za.view(B * T, D), zb.view(B * T, D)
        Cm = torch.empty(D, D, device=z_a.device, dtype=F32)
        ops.gemm(za2, zb2, Cm, D, D, B * T, a_kc=False, b_kc=False, lda=D, ldb=D, ldc=D, alpha=1.0 / (N * T))
        if group is not None:
            dist.all_reduce(Cm, group=group)
        loss = ops.lfd_loss(Cm, lam)
        ctx.save_for_backward(za, zb, isa, isb, Cm)
        ctx.args = (B, T, D, lam, N, W, group)
        return loss

    @staticmethod
    def backward(ctx, g):
        za, zb, isa, isb, Cm = ctx.saved_tensors
        B, T, D, lam, N, W, group = ctx.args
        cd = rt.compute_dtype()
        dC = ops.lfd_dloss(Cm, g.reshape(1).to(F32).contiguous(), lam, cd)
        za2, zb2 = za.view(B * T, D), zb.view(B * T, D)
        dza = torch.empty(B * T, D, device=za.device, dtype=F32)
        dzb = torch.empty(B * T, D, device=za.device, dtype=F32)
        # dza~[n][i] = sum_j dC[i][j] zb~[n][j] / NT ;  dzb~[n][j] = sum_i za~[n][i] dC[i][j] / NT
        ops.gemm(zb2, dC, dza, B * T, D, D, a_kc=True, b_kc=True, lda=D, ldb=D, ldc=D, alpha=1.0 / (N * T))
        ops.gemm(za2, dC, dzb, B * T, D, D, a_kc=True, b_kc=False, lda=D, ldb=D, ldc=D, alpha=1.0 / (N * T))
        if group is None:
            ga = ops.lfd_std_bwd(dza.view(B, T * D), za, isa).view(B, T, D)
            gb = ops.lfd_std_bwd(dzb.view(B, T * D), zb, isb).view(B, T, D)
        else:
            import torch.distributed as dist
            C = T * D
            sums = torch.empty(4 * C, device=za.device, dtype=F32)
            ops.lfd_bwd_colstat(dza.view(B, C), za, sums[:2 * C])
            ops.lfd_bwd_colstat(dzb.view(B, C), zb, sums[2 * C:])
            dist.all_reduce(sums, group=group)
            ga = ops.lfd_std_bwd_apply(dza.view(B, C), za, isa, sums[:2 * C], 1.0 / N, float(W)).view(B, T, D)
            gb = ops.lfd_std_bwd_apply(dzb.view(B, C), zb, isb, sums[2 * C:], 1.0 / N, float(W)).view(B, T, D)
        return ga, gb, None, None, None
