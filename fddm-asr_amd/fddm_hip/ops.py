"""Thin torch-tensor wrappers over libfddm_hip (one function per C entry point, plus shape helpers).

Every wrapper launches on torch's current HIP stream and checks the hipError_t. Tensors must be
contiguous where the kernel assumes it; shapes are validated here before any launch so a kernel
never sees operands that disagree with its grid.
"""
from __future__ import annotations

import math
import os

import torch

from ._lib import call, lib

F32, BF16 = 0, 1
EPI_STORE, EPI_GELU, EPI_ACC, EPI_GELU_ONLY, EPI_DGELU = 0, 1, 2, 3, 4


def code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"unsupported dtype {t.dtype}")


def tdtype(c: int):
    return torch.float32 if c == F32 else torch.bfloat16


def ptr(t):
    return 0 if t is None else t.data_ptr()


_raw_stream = torch._C._cuda_getCurrentRawStream
_cur_device = torch._C._cuda_getDevice


def stream():
    """The current HIP stream of the current device as a raw handle (the launch path's hottest host call:
    torch.cuda.current_stream() builds a Stream object and resolves the device index through Python)."""
    return _raw_stream(_cur_device())


def _chk(cond, msg):
    if not cond:
        raise ValueError(msg)


# ------------------------------------------------------------------------------------------ GEMM
def _layout_ok(A, B, M, N, K, a_kc, b_kc, lda, ldb):
    """fddm_gemm's layout preconditions (csrc/gemm.hip): 16-B chunks of every operand row never straddle a row end
    (the contiguous dimension of each operand and its leading dimension are multiples of 8 bf16 / 4 f32 elements)
    and both operand base addresses are 16-B aligned."""
    ech = 8 if B.dtype == torch.bfloat16 else 4
    ok = (K % ech == 0 if a_kc else M % ech == 0) and lda % ech == 0
    ok = ok and (K % ech == 0 if b_kc else N % ech == 0) and ldb % ech == 0
    return ok and A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0


def _gemm_padded(A, B, C, M, N, K, a_kc, b_kc, lda, ldb, ldc, epi, bias, alpha, colsum):
    """A GEMM whose operands miss the kernels' layout preconditions (a vocabulary or width that is not a multiple of
    8, e.g. the head / TextEmbedding GEMMs at V % 8 != 0): the operands are copied into zero-padded buffers (M, N,
    K rounded up to 8; the zero tail adds nothing to any dot product), the padded GEMM runs, and the M x N block is
    copied back. STORE / ACCUMULATE epilogues with bias and the fused column sum only."""
    _chk(epi in (EPI_STORE, EPI_ACC), "ragged GEMM: only store / accumulate epilogues have a padded form")
    p8 = lambda n: (n + 7) // 8 * 8   # noqa: E731
    Mp, Np, Kp = p8(M), p8(N), p8(K)
    a = torch.as_strided(A, (M, K) if a_kc else (K, M), (lda, 1))
    b = torch.as_strided(B, (N, K) if b_kc else (K, N), (ldb, 1))
    Ap = torch.zeros((Mp, Kp) if a_kc else (Kp, Mp), device=A.device, dtype=A.dtype)
    Bp = torch.zeros((Np, Kp) if b_kc else (Kp, Np), device=B.device, dtype=B.dtype)
    Ap[: a.shape[0], : a.shape[1]] = a
    Bp[: b.shape[0], : b.shape[1]] = b
    c = torch.as_strided(C, (M, N), (ldc, 1))
    Cp = torch.zeros(Mp, Np, device=C.device, dtype=C.dtype)
    if epi == EPI_ACC:
        Cp[:M, :N] = c
    bp = None
    if bias is not None:
        bp = torch.zeros(Np, device=bias.device, dtype=bias.dtype)
        bp[:N] = bias[:N]
    cs = None
    if colsum is not None:
        cs = torch.zeros(Mp, device=colsum.device, dtype=colsum.dtype)
        if epi == EPI_ACC:
            cs[:M] = colsum[:M]
    gemm(Ap, Bp, Cp, Mp, Np, Kp, a_kc=a_kc, b_kc=b_kc, lda=Ap.shape[1], ldb=Bp.shape[1], ldc=Np, epi=epi, bias=bp,
         alpha=alpha, colsum=cs)
    c.copy_(Cp[:M, :N])
    if colsum is not None:
        colsum[:M].copy_(cs[:M])
    return C


GEMM_PATHS = {"auto": 0, "big": 1, "small": 2, "256": 3, "128": 4}


def gemm_force_path(name: str) -> str:
    """Force a GEMM kernel family for every following fddm_gemm / conv GEMM launch (tests and diagnostics; "auto"
    restores the shape-based choice). Returns the previous setting's name."""
    from ._lib import lib
    old = lib().fddm_gemm_force_path(GEMM_PATHS[name])     # returns the previous path, not an error code
    return {v: k for k, v in GEMM_PATHS.items()}[old]


ATTN_KERNELS = {"auto": 0, "v6": 1, "nofused": 2, "fwd7": 3, "fwd8": 4, "relfwd5": 5}


def attn_force_kernels(name: str) -> str:
    """Select the attention kernel family for every following launch (tests and diagnostics): "v6" = the
    16x16x32-MFMA kernels of attention.hip where the 32x32x16 family (attn7.hip) would run, "nofused" = the 32x32x16
    family without its fused backward (dq7 + dkv7 at every key length), "fwd7" = the default with the one-chain forward
    fwd7 everywhere, "fwd8" = the default with the two-chain fwd8 (attn8.hip) everywhere, "relfwd5" = the default with
    WavLM's biased attention on the round-2 fwd5 instead of fwd7's REL build, "auto" = the default choice (fwd8 unless
    its 256-query workgroups load the busiest CU with more queries than fwd7's). Returns the previous setting's name."""
    from ._lib import lib
    old = lib().fddm_attn_set_kernels(ATTN_KERNELS[name])
    return {v: k for k, v in ATTN_KERNELS.items()}[old]


def gemm(A, B, C, M, N, K, *, a_kc=True, b_kc=True, lda, ldb, ldc, epi=EPI_STORE, bias=None, alpha=1.0,
         C2=None, Mi=0, sAb=0, drop_p=0.0, seed=0, rng_stream=0, colsum=None):
    """C[m][n] = alpha * sum_k A(m,k) B(n,k) (+bias, epilogue). Compute dtype = B.dtype.
    Operands that miss the kernels' layout preconditions (a dimension or leading dimension not a multiple of 8, e.g.
    a ragged vocabulary) run zero-padded copies (_gemm_padded) — unbatched calls only: a batched / strided call
    (Mi or sAb set) with such operands raises."""
    _chk(B.dtype in (torch.float32, torch.bfloat16), "B dtype")
    if M == 0 or N == 0:
        return C
    if not _layout_ok(A, B, M, N, K, a_kc, b_kc, lda, ldb):
        _chk(Mi == 0 and sAb == 0, "batched / strided GEMM operands must meet the 8-element layout preconditions "
                                   "(the zero-padded fallback covers unbatched calls only)")
        return _gemm_padded(A, B, C, M, N, K, a_kc, b_kc, lda, ldb, ldc, epi, bias, alpha, colsum)
    call("fddm_gemm", code(B), code(A), int(a_kc), int(b_kc), epi, code(C), ptr(A), lda, Mi, sAb, ptr(B), ldb,
         ptr(C), ldc, ptr(C2), ptr(bias), float(alpha), M, N, K, seed, rng_stream, float(drop_p), ptr(colsum),
         stream())
    return C


def linear(x2d, w, bias=None, out_dtype=None, out=None, epi=EPI_STORE, C2=None, drop_p=0.0, seed=0, rng_stream=0):
    """y[M,N] = x[M,K] @ w[N,K]^T + bias.  x, w: compute dtype (x may be f32 when w is bf16)."""
    M, K = x2d.shape
    N = w.shape[0]
    _chk(w.shape[1] == K and x2d.stride(1) == 1 and w.is_contiguous(), "linear shapes")
    if out is None:
        out = torch.empty(M, N, device=x2d.device, dtype=out_dtype or w.dtype)
    return gemm(x2d, w, out, M, N, K, lda=x2d.stride(0), ldb=K, ldc=out.stride(0), epi=epi, bias=bias, C2=C2,
                drop_p=drop_p, seed=seed, rng_stream=rng_stream)


def linear_dx(dy2d, w, out=None, accumulate=False, out_dtype=torch.float32, epi=None, C2=None, drop_p=0.0, seed=0,
              rng_stream=0):
    """dx[M,K] = dy[M,N] @ w[N,K]  (w M/N-contiguous operand). accumulate -> out (f32) += ."""
    M, N = dy2d.shape
    K = w.shape[1]
    _chk(w.shape[0] == N and w.is_contiguous() and dy2d.stride(1) == 1, "linear_dx shapes")
    if out is None:
        out = torch.empty(M, K, device=dy2d.device, dtype=out_dtype)
    e = EPI_ACC if accumulate else (EPI_STORE if epi is None else epi)
    return gemm(dy2d, w, out, M, K, N, a_kc=True, b_kc=False, lda=dy2d.stride(0), ldb=K, ldc=out.stride(0), epi=e,
                C2=C2, drop_p=drop_p, seed=seed, rng_stream=rng_stream)


_NO_ROPE_FUSE = os.environ.get("FDDM_ROPE_FUSE", "1") == "0"     # diagnostic A/B knob (tools/ab.sh)


def linear_dx_rope(dy2d, w, dx, cs, sn, L) -> bool:
    """dx[M,d] += rope_bwd(dy[M,n] @ w[n,d]) in one launch (fddm_linear_dx_rope: the self-attention input gradient
    through RoPE). Returns False, launching nothing, where the fused kernel does not apply (not bf16, d % 128 != 0,
    a GEMM-family override): the caller then runs linear_dx into a temporary + rope_bwd."""
    M, N = dy2d.shape
    d = w.shape[1]
    if _NO_ROPE_FUSE:
        return False
    if not (dy2d.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and dx.dtype == torch.float32 and d % 128 == 0
            and w.shape[0] == N and w.is_contiguous() and dy2d.stride(1) == 1 and dx.is_contiguous()
            and cs.is_contiguous() and sn.is_contiguous() and cs.dtype == torch.float32 and cs.shape[-1] == d):
        return False
    rc = lib().fddm_linear_dx_rope(ptr(dy2d), dy2d.stride(0), ptr(w), d, ptr(dx), d, ptr(cs), ptr(sn), M, d, N, L,
                                   stream())
    if rc == 1:      # hipErrorInvalidValue: not applicable, nothing launched
        return False
    if rc != 0:
        msg = lib().fddm_error_string(rc)
        raise RuntimeError(f"fddm_linear_dx_rope failed: hipError {rc} ({msg.decode() if msg else '?'})")
    return True


def linear_dw(dy2d, x2d, out=None, accumulate=False, db=None):
    """dW[N,K] = dy[M,N]^T @ x[M,K]  (both M/N-contiguous operands, K-reduction over tokens);
    db (optional, f32 [N]) receives sum_m dy[m] — the bias gradient, fused into the same launch.
    accumulate: out += and db += (grad-arena slots); otherwise both are overwritten."""
    M, N = dy2d.shape
    K = x2d.shape[1]
    _chk(x2d.shape[0] == M and dy2d.stride(1) == 1 and x2d.stride(1) == 1, "linear_dw shapes")
    if out is None:
        out = torch.empty(N, K, device=dy2d.device, dtype=torch.float32)
    if db is not None and dy2d.dtype != x2d.dtype:
        gemm(dy2d, x2d, out, N, K, M, a_kc=False, b_kc=False, lda=dy2d.stride(0), ldb=x2d.stride(0),
             ldc=out.stride(0), epi=EPI_ACC if accumulate else EPI_STORE)
        colsum(dy2d, out=db, accumulate=accumulate)
        return out
    return gemm(dy2d, x2d, out, N, K, M, a_kc=False, b_kc=False, lda=dy2d.stride(0), ldb=x2d.stride(0),
                ldc=out.stride(0), epi=EPI_ACC if accumulate else EPI_STORE, colsum=db)


def linear_dw_grouped(jobs, kchunk=0):
    """One launch for several weight-gradient GEMMs, all accumulating: for each (dy [K,M], x [K,N], dW [M,N] f32,
    db [M] f32 or None): dW += dy^T x, db += sum_k dy. dy/x bf16 with unit inner stride.
    kchunk 0: the library balances split-K over the CUs (128x128 LDS-DMA kernel); kchunk > 0: every workgroup
    of the 128x128 register-staged kernel reduces about kchunk tokens."""
    import ctypes
    jobs = [j for j in jobs if j[0].shape[0] > 0]
    for i in range(0, len(jobs), 12):
        chunk = jobs[i:i + 12]
        n = len(chunk)
        for dy, x, dW, db in chunk:
            _chk(dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and dW.dtype == torch.float32, "dw dtypes")
            _chk(dy.shape[0] == x.shape[0] and dW.shape == (dy.shape[1], x.shape[1]), "dw shapes")
            _chk(dy.stride(1) == 1 and x.stride(1) == 1 and dW.stride(1) == 1, "dw strides")
            _chk(db is None or (db.dtype == torch.float32 and db.is_contiguous() and db.numel() == dy.shape[1]),
                 "db")
        P = ctypes.c_void_p * n
        L = ctypes.c_long * n
        call("fddm_gemm_dw_grouped", n, P(*[j[0].data_ptr() for j in chunk]), L(*[j[0].stride(0) for j in chunk]),
             P(*[j[1].data_ptr() for j in chunk]), L(*[j[1].stride(0) for j in chunk]),
             P(*[j[2].data_ptr() for j in chunk]), L(*[j[2].stride(0) for j in chunk]),
             P(*[ptr(j[3]) for j in chunk]), L(*[j[0].shape[1] for j in chunk]), L(*[j[1].shape[1] for j in chunk]),
             L(*[j[0].shape[0] for j in chunk]), kchunk, stream())


def colsum(X2d, out=None, accumulate=False):
    M, N = X2d.shape
    if out is None:
        out = torch.zeros(N, device=X2d.device, dtype=torch.float32)
    elif not accumulate:
        out.zero_()
    call("fddm_colsum", code(X2d), ptr(X2d), ptr(out), M, N, X2d.stride(0), stream())
    return out


def conv1d_gemm(x, W, out, *, lda, sAb, Tin, Cg, cstride, cpad, Bn, Tout, N, K, groups=1, bias=None, gelu=False):
    call("fddm_conv1d_gemm", code(W), EPI_GELU_ONLY if gelu else EPI_STORE, ptr(x), lda, sAb, Tin, Cg, cstride,
         cpad, ptr(W), ptr(out), out.shape[-1], ptr(bias), Bn, Tout, N, K, groups, stream())
    return out


def posconv_gelu(x, W, bias, out, B, S, E, G, kp):
    """WavLM positional conv + GELU (bf16): x/out [B*S, E], W [G, Cg, kp*Cg], bias [E] f32."""
    _chk(x.dtype == torch.bfloat16 and W.dtype == torch.bfloat16 and out.dtype == torch.bfloat16, "posconv dtypes")
    _chk(x.is_contiguous() and W.is_contiguous() and out.is_contiguous() and bias.is_contiguous(), "posconv layout")
    _chk(x.numel() == B * S * E and out.numel() == B * S * E and W.numel() == E * kp * (E // G), "posconv shapes")
    call("fddm_posconv_gelu", ptr(x), ptr(W), ptr(bias), ptr(out), B, S, E, G, kp, stream())
    return out


def conv0_gn_gelu(wave, w, gamma, beta, out_dtype, C, K, S, eps=1e-5):
    B, nsamp = wave.shape
    T0 = (nsamp - K) // S + 1
    nb = (T0 + 4095) // 4096  # statistics blocks per utterance (wavlm.hip C0_GRAM_FRAMES)
    ws = torch.empty(B * nb * (K + K * (K + 1) // 2) + B * C, device=wave.device, dtype=torch.float64)
    out = torch.empty(B, T0, C, device=wave.device, dtype=out_dtype)
    call("fddm_conv0_gn_gelu", code(out), ptr(wave), ptr(w), ptr(gamma), ptr(beta), ptr(ws), ptr(out), B, nsamp, T0,
         C, K, S, float(eps), stream())
    return out


def wavlm_gate(x2d, W, bias, cst, B, S, H):
    E = x2d.shape[1]
    gate = torch.empty(B * H, S, device=x2d.device, dtype=torch.float32)
    call("fddm_wavlm_gate", code(x2d), ptr(x2d), ptr(W), ptr(bias), ptr(cst), ptr(gate), B, S, H, E, stream())
    return gate


# ------------------------------------------------------------------------------------- attention
def drop_words(B, H, Lq, Lk):
    """u64 words per site of a keep-bit buffer (fddm_attn_drop_words: room for either storage layout)."""
    from ._lib import lib
    return int(lib().fddm_attn_drop_words(B, H, Lq, Lk))


def drop_bits(B, H, Lq, Lk, device):
    """Buffer for one attention site's dropout keep bits (written by attn_drop_bits or by the forward, read by the
    backward; the layout is the selected kernel family's: csrc/attn7.hip layout v3 by default)."""
    return torch.empty(drop_words(B, H, Lq, Lk), device=device, dtype=torch.int64)


def _heads(x, rows, H, dh):
    """[rows, H*dh] view (any row stride) as [rows, H, dh]."""
    return x[:rows, : H * dh].unflatten(1, (H, dh))


def _pad64(x, rows, H, dh):
    """Head slots widened to the kernels' 64 lanes with zeros: [rows, H*64]. Zero q/k columns add nothing to
    Q K^T and zero v columns give zero output columns, so the attention of the first dh columns is unchanged."""
    xp = torch.zeros(rows, H, 64, device=x.device, dtype=x.dtype)
    xp[:, :, :dh] = _heads(x, rows, H, dh)
    return xp.view(rows, H * 64)


def attn_drop_bits(out, nsites, B, H, Lq, Lk, drop_p, seed, stream0, stream_step):
    """The dropout keep-bit words of `nsites` attention sites of one shape (rng streams stream0 + s * stream_step)
    into out [nsites, words] (int64): what attn_fwd(..., dbits=out[s], bits_ready=True) and attn_bwd read."""
    _chk(out.dtype == torch.int64 and out.is_contiguous() and out.dim() == 2 and out.shape[0] >= nsites,
         "drop-bit buffer layout")
    call("fddm_attn_drop_bits", ptr(out), out.shape[1], nsites, B, H, Lq, Lk, float(drop_p), seed, stream0,
         stream_step, stream())
    return out


def attn_fwd(q, k, v, out, lse, B, H, Lq, Lk, *, key_keep=None, gate=None, table=None, drop_p=0.0, seed=0,
             rng_stream=0, scale=None, dbits=None, bits_ready=False):
    """q: [B*Lq, >=H*dh] row stride q.stride(0); k/v: [B*Lk, ...]; out [B*Lq, H*dh]; lse [B*H, Lq], dh =
    out.shape[1] // H. dbits (optional, drop_bits()): the dropout keep bits the backward reads; bits_ready: they
    were already written by attn_drop_bits (the forward only reads them), else the forward writes them.
    The kernels are built for head_dim 64; a smaller head_dim (the reference's nn.MultiheadAttention takes any
    d_model / nhead) runs them on zero-padded 64-wide head slots — the scores, the softmax, the dropout
    element indices (b, h, query, key) and hence the RNG stream are those of the unpadded heads."""
    _chk(q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1, "attention inputs need unit inner stride")
    _chk(q.dtype == k.dtype == v.dtype == out.dtype, "attention dtype mismatch")
    _chk(out.shape[1] % H == 0, "attention output width must be H * head_dim")
    dh = out.shape[1] // H
    _chk(1 <= dh <= 64, f"head_dim {dh} > 64 is not built")
    sc = 1.0 / math.sqrt(dh) if scale is None else scale
    if dh != 64:
        op = torch.empty(B * Lq, H * 64, device=out.device, dtype=out.dtype)
        attn_fwd(_pad64(q, B * Lq, H, dh), _pad64(k, B * Lk, H, dh), _pad64(v, B * Lk, H, dh), op, lse, B, H, Lq,
                 Lk, key_keep=key_keep, gate=gate, table=table, drop_p=drop_p, seed=seed, rng_stream=rng_stream,
                 scale=sc, dbits=dbits, bits_ready=bits_ready)
        _heads(out, B * Lq, H, dh).copy_(op.view(B * Lq, H, 64)[:, :, :dh])
        return out
    call("fddm_attn_fwd", code(q), ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out),
         out.stride(0), ptr(lse), ptr(key_keep), ptr(gate), ptr(table), B, H, Lq, Lk, float(sc), float(drop_p), seed,
         rng_stream, ptr(dbits), int(bool(bits_ready) and dbits is not None), stream())
    return out


def attn_fwd_relgate_x(q, k, v, out, x, gw, gconst, table, B, H, L, scale=None):
    """WavLM attention (bf16) with the gate computed in the kernel from the attention input x [B*L, H*64] (bf16, row
    stride x.stride(0)) and the folded gru_rel_pos_linear weights gw (130 floats: sum of weight rows 0-3, rows 4-7,
    the two bias sums; models/wavlm.py)."""
    _chk(q.dtype == k.dtype == v.dtype == out.dtype == x.dtype == torch.bfloat16, "relgate attention is bf16")
    _chk(x.stride(-1) == 1 and x.shape[1] >= H * 64 and x.data_ptr() % 16 == 0, "gate input layout")
    _chk(gw.dtype == torch.float32 and gw.numel() >= 130 and gw.is_contiguous() and gw.data_ptr() % 16 == 0,
         "folded gate weights")
    sc = 1.0 / math.sqrt(64) if scale is None else scale
    call("fddm_attn_fwd_relgate_x", ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out),
         out.stride(0), ptr(x), x.stride(0), ptr(gw), ptr(gconst), ptr(table), B, H, L, L, float(sc), stream())
    return out


def attn_fwd_relgate(q, k, v, out, graw, gconst, table, B, H, L, scale=None):
    """WavLM attention (bf16) with the gate computed in the kernel from graw [B*L, >= H*8] (row stride
    graw.stride(0)): 8 gru_rel_pos_linear pre-activations per (token, head)."""
    _chk(q.dtype == k.dtype == v.dtype == out.dtype == graw.dtype == torch.bfloat16, "relgate attention is bf16")
    _chk(graw.stride(-1) == 1 and graw.shape[1] >= H * 8 and graw.data_ptr() % 16 == 0, "graw layout")
    sc = 1.0 / math.sqrt(64) if scale is None else scale
    call("fddm_attn_fwd_relgate", ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out),
         out.stride(0), ptr(graw), graw.stride(0), ptr(gconst), ptr(table), B, H, L, L, float(sc), stream())
    return out


def attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, *, key_keep=None, drop_p=0.0, seed=0, rng_stream=0,
             dbits=None, scale=None):
    """Gradients of attn_fwd (same layouts; head_dim = o.shape[1] // H, padded to 64 as in attn_fwd)."""
    _chk(o.shape[1] % H == 0, "attention output width must be H * head_dim")
    dh = o.shape[1] // H
    _chk(1 <= dh <= 64, f"head_dim {dh} > 64 is not built")
    sc = 1.0 / math.sqrt(dh) if scale is None else scale
    if dh != 64:
        rq, rk = B * Lq, B * Lk
        dqp = torch.empty(rq, H * 64, device=dq.device, dtype=dq.dtype)
        dkp = torch.empty(rk, H * 64, device=dk.device, dtype=dk.dtype)
        dvp = torch.empty(rk, H * 64, device=dv.device, dtype=dv.dtype)
        attn_bwd(_pad64(q, rq, H, dh), _pad64(k, rk, H, dh), _pad64(v, rk, H, dh), _pad64(o, rq, H, dh),
                 _pad64(do, rq, H, dh), lse, dqp, dkp, dvp, B, H, Lq, Lk, key_keep=key_keep, drop_p=drop_p, seed=seed,
                 rng_stream=rng_stream, dbits=dbits, scale=sc)
        for g, gp, r in ((dq, dqp, rq), (dk, dkp, rk), (dv, dvp, rk)):
            _heads(g, r, H, dh).copy_(gp.view(r, H, 64)[:, :, :dh])
        return
    # row-term workspace: delta = rowsum(dO O) and -LSE log2(e) per query, [2][B*H][Lq rounded up to 64] (the
    # 32x32x16 backward's layout; the other kernels use the first B*H*Lq floats)
    delta = torch.empty(int(lib().fddm_attn_bwd_ws_floats(B, H, Lq, Lk)), device=q.device, dtype=torch.float32)
    call("fddm_attn_bwd", code(q), ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(o),
         o.stride(0), ptr(do), do.stride(0), ptr(lse), ptr(dq), dq.stride(0), ptr(dk), dk.stride(0), ptr(dv),
         dv.stride(0), ptr(delta), ptr(key_keep), B, H, Lq, Lk, float(sc), float(drop_p), seed, rng_stream,
         ptr(dbits), stream())


# ----------------------------------------------------------------------------------- layernorm
def ln_fwd(x, y, gamma, beta, *, out_f32=None, out_t=None, save_s=None, mean=None, rstd=None, film=None,
           rows_per_batch=0, eps=1e-5, drop_p=0.0, seed=0, rng_stream=0, rope=None):
    """rope = (cos [L, d], sin [L, d], out bf16 [N, d], L): also write RoPE(output) — rope_fwd of the output — for the
    decoder's next block (f32 x, bf16 y and out_t, no FiLM)."""
    N, d = x.shape
    fs, fh = film if film is not None else (None, None)
    rc, rs, ro, rl = rope if rope is not None else (None, None, None, 0)
    out_code = code(out_t) if out_t is not None else code(x if y is None else y)
    ycode = code(y) if y is not None else code(x)
    call("fddm_ln_fwd", code(x), ycode, out_code, ptr(x), ptr(y), ptr(gamma), ptr(beta), ptr(fs), ptr(fh),
         ptr(out_f32), ptr(out_t), ptr(save_s), ptr(mean), ptr(rstd), N, d, rows_per_batch, float(eps), float(drop_p),
         seed, rng_stream, ptr(rc), ptr(rs), ptr(ro), rl, stream())


def ln_bwd(dout, s, mean, rstd, gamma, beta, *, dres=None, dy_t=None, dgamma=None, dbeta=None, film_scale=None,
           dfilm=None, rows_per_batch=0, drop_p=0.0, seed=0, rng_stream=0, partials=None):
    """partials: a LnPartials (ln_partials) collecting this LayerNorm's dgamma / dbeta slab sums for one ln_fold launch
    (the fused pass only), or None: the sums are added to dgamma / dbeta with atomics."""
    N, d = dout.shape
    dfs, dfh = dfilm if dfilm is not None else (None, None)
    part = None
    if partials is not None:
        _chk(dgamma is not None and dbeta is not None, "ln_bwd partials need dgamma and dbeta")
        part = partials.add(N, d, dgamma, dbeta, (dfs, dfh) if film_scale is not None else None, rows_per_batch)
    call("fddm_ln_bwd", code(dy_t) if dy_t is not None else F32, ptr(dout), ptr(s), ptr(mean), ptr(rstd), ptr(gamma),
         ptr(beta), ptr(film_scale), ptr(dres), ptr(dy_t), ptr(dgamma), ptr(dbeta), ptr(dfs), ptr(dfh), N, d,
         rows_per_batch, float(drop_p), seed, rng_stream, ptr(part), stream())


class LnPartials:
    """The dgamma / dbeta slab sums of up to 4 LayerNorm backwards (ln_bwd(partials=...)), added to their
    destinations by one ln_fold launch: the slab atomics of ~5 us per LayerNorm backward become one short fold."""

    def __init__(self):
        self.jobs = []

    def add(self, N, d, dgamma, dbeta, dfilm=None, rows_per_batch=0):
        """dfilm = (dfs, dfh) [B, d] with FiLM batches of rows_per_batch rows: folded per batch when the batches
        are whole slabs (the fused pass); otherwise the backward adds them with atomics and leaves zeros here."""
        _chk(len(self.jobs) < 4, "at most 4 LayerNorms per fold")
        rows = lib().fddm_ln_bwd_slab_rows()
        nslab = (N + rows - 1) // rows
        part = torch.empty(nslab, 4, d, device=dgamma.device, dtype=torch.float32)
        dfs = dfh = None
        spb = 0
        if dfilm is not None and rows_per_batch > 0 and rows_per_batch % rows == 0:
            dfs, dfh = dfilm
            spb = rows_per_batch // rows
        self.jobs.append((part, nslab, d, dgamma, dbeta, dfs, dfh, spb))
        return part

    def fold(self):
        import ctypes
        n = len(self.jobs)
        if n == 0:
            return
        P = ctypes.c_void_p * n
        Lg = ctypes.c_long * n
        J = self.jobs
        call("fddm_ln_fold", n, P(*[j[0].data_ptr() for j in J]), Lg(*[j[1] for j in J]), Lg(*[j[2] for j in J]),
             P(*[j[3].data_ptr() for j in J]), P(*[j[4].data_ptr() for j in J]), P(*[ptr(j[5]) for j in J]),
             P(*[ptr(j[6]) for j in J]), Lg(*[j[7] for j in J]), stream())
        self.jobs = []


# -------------------------------------------------------------------------------- small kernels
def rope_fwd(x, cs, sn, out, L):
    N, d = x.shape
    call("fddm_rope_fwd", code(out), ptr(x), ptr(cs), ptr(sn), ptr(out), N, L, d, stream())
    return out


def rope_bwd(dy, cs, sn, dx, L):
    N, d = dy.shape
    call("fddm_rope_bwd", ptr(dy), ptr(cs), ptr(sn), ptr(dx), N, L, d, stream())


def embed_fwd(tok, E, tbias, out, out_t, L):
    N = tok.numel()
    d = E.shape[1]
    call("fddm_embed_fwd", code(out_t) if out_t is not None else F32, ptr(tok), ptr(E), ptr(tbias), ptr(out),
         ptr(out_t), N, L, d, stream())


def embed_bwd(tok, dx, dE, dtb, L, pad_id):
    N, d = dx.shape
    call("fddm_embed_bwd", ptr(tok), ptr(dx), ptr(dE), ptr(dtb), N, L, d, pad_id, stream())


def cast(x, dtype, out=None):
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=dtype)
    call("fddm_cast", code(x), code(out), ptr(x), ptr(out), x.numel(), stream())
    return out


def sample_q(x0, t, thr, K, seed, rng_stream=1):
    B, L = x0.shape
    xt = torch.empty_like(x0)
    call("fddm_sample_q", ptr(x0), ptr(t), ptr(thr), ptr(xt), B, L, K, seed, rng_stream, stream())
    return xt


def kl_fwd(logits2d, xt, x0, t, betas, L):
    N, V = logits2d.shape
    kl = torch.empty(N, device=logits2d.device, dtype=torch.float32)
    call("fddm_kl_fwd", ptr(logits2d), ptr(xt), ptr(x0), ptr(t), ptr(betas), ptr(kl), N, L, V, stream())
    return kl


def kl_bwd(logits2d, xt, x0, t, betas, w, gscale, L, out_dtype=torch.float32):
    N, V = logits2d.shape
    dz = torch.empty(N, V, device=logits2d.device, dtype=out_dtype)
    call("fddm_kl_bwd", ptr(logits2d), ptr(xt), ptr(x0), ptr(t), ptr(betas), ptr(w), ptr(gscale), ptr(dz),
         code(dz), N, L, V, stream())
    return dz


KL_FUSED_MAX_V = 32768      # fddm_kl_fused: 512 threads x 16 float4 per row


def kl_fused(logits2d, xt, x0, t, betas, mask_u8, L, out_dtype=torch.float32):
    """(kl_tok [N] f32, dz [N, V]) in one pass: dz = w * d kl_tok / d logits with kl_reduce's weights w (from the
    uint8 mask [N], or None = plain mean over L); the upstream gradient is applied later by scale_if."""
    N, V = logits2d.shape
    _chk(logits2d.dtype == torch.float32 and logits2d.is_contiguous() and N % L == 0, "kl_fused: f32 [B*L, V] rows")
    _chk(mask_u8 is None or (mask_u8.numel() == N and mask_u8.dtype == torch.uint8), "kl_fused mask")
    kl = torch.empty(N, device=logits2d.device, dtype=torch.float32)
    dz = torch.empty(N, V, device=logits2d.device, dtype=out_dtype)
    call("fddm_kl_fused", ptr(logits2d), ptr(xt), ptr(x0), ptr(t), ptr(betas), ptr(mask_u8), ptr(kl), ptr(dz),
         code(dz), N, L, V, stream())
    return kl, dz


def scale_if(x, g):
    """x *= g (a device scalar), in place; no memory traffic when g == 1."""
    _chk(x.is_contiguous() and g.dtype == torch.float32 and g.numel() == 1, "scale_if operands")
    call("fddm_scale_if", ptr(x), code(x), ptr(g), x.numel(), stream())
    return x


def softmax_bwd_add_bf16(y, dy, add, out=None):
    """out = bf16(y * (dy - rowsum(y*dy)) + add), all bf16 [N, V] (out may be `add`)."""
    N, V = y.shape
    _chk(all(t.dtype == torch.bfloat16 and t.is_contiguous() and tuple(t.shape) == (N, V) for t in (y, dy, add)),
         "softmax_bwd_add_bf16 operands")
    if out is None:
        out = torch.empty_like(y)
    call("fddm_softmax_bwd_add_bf16", ptr(y), ptr(dy), ptr(add), ptr(out), N, V, stream())
    return out


def axpy_if_bf16(x, y, g):
    """x += (g - 1) * y in place (bf16), no memory traffic when the device scalar g == 1."""
    _chk(x.dtype == y.dtype == torch.bfloat16 and x.numel() == y.numel() and x.is_contiguous() and y.is_contiguous(),
         "axpy_if_bf16 operands")
    call("fddm_axpy_if_bf16", ptr(x), ptr(y), ptr(g), x.numel(), stream())
    return x


def softmax_rows(x2d, out_dtype):
    N, V = x2d.shape
    y = torch.empty(N, V, device=x2d.device, dtype=out_dtype)
    call("fddm_softmax_rows", ptr(x2d), ptr(y), code(y), N, V, stream())
    return y


def softmax_bwd_rows(y, dy, dz=None, accumulate=False):
    N, V = y.shape
    if dz is None:
        dz = torch.empty(N, V, device=y.device, dtype=torch.float32)
    call("fddm_softmax_bwd_rows", ptr(y), ptr(dy), ptr(dz), code(y), N, V, int(accumulate), stream())
    return dz


def lfd_std_fwd(z2d, out_dtype, eps=1e-5):
    B, C = z2d.shape
    zt = torch.empty(B, C, device=z2d.device, dtype=out_dtype)
    inv_std = torch.empty(C, device=z2d.device, dtype=torch.float32)
    call("fddm_lfd_std_fwd", code(zt), ptr(z2d), ptr(zt), ptr(inv_std), B, C, float(eps), stream())
    return zt, inv_std


def lfd_std_bwd(dzt, zt, inv_std):
    B, C = dzt.shape
    dz = torch.empty(B, C, device=dzt.device, dtype=torch.float32)
    call("fddm_lfd_std_bwd", code(zt), ptr(dzt), ptr(zt), ptr(inv_std), ptr(dz), B, C, stream())
    return dz


def lfd_colstat(z2d, out, mean_sum=None, inv_n=0.0):
    B, C = z2d.shape
    _chk(out.numel() >= C and out.dtype == torch.float32, "lfd_colstat out")
    call("fddm_lfd_colstat", ptr(z2d), ptr(out), ptr(mean_sum), float(inv_n), B, C, stream())
    return out


def lfd_std_apply(z2d, out_dtype, s1, s2, inv_n, eps=1e-5):
    B, C = z2d.shape
    zt = torch.empty(B, C, device=z2d.device, dtype=out_dtype)
    inv_std = torch.empty(C, device=z2d.device, dtype=torch.float32)
    call("fddm_lfd_std_apply", code(zt), ptr(z2d), ptr(zt), ptr(inv_std), ptr(s1), ptr(s2), float(inv_n), float(eps), B,
         C, stream())
    return zt, inv_std


def lfd_bwd_colstat(dzt, zt, out):
    B, C = dzt.shape
    _chk(out.numel() >= 2 * C and out.dtype == torch.float32, "lfd_bwd_colstat out")
    call("fddm_lfd_bwd_colstat", code(zt), ptr(dzt), ptr(zt), ptr(out), B, C, stream())
    return out


def lfd_std_bwd_apply(dzt, zt, inv_std, sums, inv_n, scale=1.0):
    B, C = dzt.shape
    dz = torch.empty(B, C, device=dzt.device, dtype=torch.float32)
    call("fddm_lfd_std_bwd_apply", code(zt), ptr(dzt), ptr(zt), ptr(inv_std), ptr(sums), float(inv_n), float(scale),
         ptr(dz), B, C, stream())
    return dz


def lfd_loss(Cm, lam):
    D = Cm.shape[0]
    loss = torch.empty((), device=Cm.device, dtype=torch.float32)
    call("fddm_lfd_loss", ptr(Cm), ptr(loss), D, float(lam), stream())
    return loss


def lfd_dloss(Cm, gscale, lam, out_dtype):
    D = Cm.shape[0]
    dC = torch.empty(D, D, device=Cm.device, dtype=out_dtype)
    call("fddm_lfd_dloss", code(dC), ptr(Cm), ptr(gscale), ptr(dC), D, float(lam), stream())
    return dC


# ----------------------------------------------------------------------------- small per-batch ops
def rows_mean(x3d):
    """[B, S, d] (f32 / bf16, contiguous) -> f32 [B, d] mean over S."""
    B, S, d = x3d.shape
    _chk(x3d.is_contiguous(), "rows_mean: contiguous input")
    out = torch.empty(B, d, device=x3d.device, dtype=torch.float32)
    call("fddm_rows_mean", code(x3d), ptr(x3d), ptr(out), B, S, d, stream())
    return out


def time_embed(t, d, max_steps):
    """SinusoidalTimeEmbedding features of int64 t [B] -> f32 [B, d]."""
    _chk(t.dtype == torch.int64 and t.is_contiguous() and t.dim() == 1, "time_embed: int64 [B]")
    emb = torch.empty(t.numel(), d, device=t.device, dtype=torch.float32)
    call("fddm_time_embed", ptr(t), ptr(emb), t.numel(), d, float(max_steps), stream())
    return emb


def _parr(ts):
    import ctypes
    return (ctypes.c_void_p * len(ts))(*[ptr(x) for x in ts])


def small_linear(inp, Ws, bs, outs, outs2=None, act=0, aux=None, transpose_w=False):
    """out_j = act(inp @ W_j^T + b_j) (transpose_w: inp @ W_j) for a few row-batch (R <= 64 per tile) fp32 Linears
    sharing one input; act 1 also writes silu into outs2; act 2 multiplies by silu'(aux)."""
    R, K = inp.shape
    W0 = Ws[0]
    N = W0.shape[0]
    if transpose_w:
        N = W0.shape[1]
        _chk(W0.shape[0] == K, "small_linear shapes")
    else:
        _chk(W0.shape[1] == K, "small_linear shapes")
    for W, o in zip(Ws, outs):
        _chk(W.dtype == torch.float32 and W.is_contiguous() and W.shape == W0.shape, "small_linear weights")
        _chk(o.dtype == torch.float32 and o.shape == (R, N) and o.stride(1) == 1 and o.stride(0) == N, "small_linear out")
    _chk(inp.dtype == torch.float32 and inp.stride(1) == 1, "small_linear input")
    ldw = W0.shape[1]
    for i in range(0, len(Ws), 16):
        sl = slice(i, i + 16)
        n = len(Ws[sl])
        call("fddm_small_linear", ptr(inp), inp.stride(0), n, _parr(Ws[sl]), _parr(bs[sl]) if bs is not None else None,
             _parr(outs[sl]), _parr(outs2[sl]) if outs2 is not None else None, ldw, N, ptr(aux), R, N, K, act,
             int(transpose_w), stream())


def small_dw(jobs):
    """For (dy [R, N], x [R, K], dW [N, K], db [N] or None): dW += dy^T x, db += colsum(dy) (fp32, R rows)."""
    import ctypes
    if not jobs:
        return
    R = jobs[0][0].shape[0]
    for dy, x, dW, db in jobs:
        _chk(dy.dtype == x.dtype == dW.dtype == torch.float32 and dy.shape[0] == x.shape[0] == R, "small_dw dtypes")
        _chk(dW.shape == (dy.shape[1], x.shape[1]) and dW.is_contiguous() and dy.stride(1) == 1 and x.stride(1) == 1,
             "small_dw shapes")
        _chk(db is None or (db.numel() == dy.shape[1] and db.is_contiguous()), "small_dw bias")
    for i in range(0, len(jobs), 16):
        ch = jobs[i:i + 16]
        L = ctypes.c_long * len(ch)
        call("fddm_small_dw", len(ch), _parr([j[0] for j in ch]), L(*[j[0].stride(0) for j in ch]),
             _parr([j[1] for j in ch]), L(*[j[1].stride(0) for j in ch]), _parr([j[2] for j in ch]),
             _parr([j[3] for j in ch]), L(*[j[0].shape[1] for j in ch]), L(*[j[1].shape[1] for j in ch]), R, stream())


def kl_reduce(kl_tok, mask_u8, B, L, want_w=True):
    """Masked batch mean of the per-token KL (train.py:247-253) -> (loss f32 scalar, w [B*L] = d loss / d kl_tok,
    or None when not wanted)."""
    _chk(kl_tok.numel() == B * L and (mask_u8 is None or (mask_u8.numel() == B * L and mask_u8.dtype == torch.uint8)),
         "kl_reduce shapes")
    loss = torch.empty((), device=kl_tok.device, dtype=torch.float32)
    w = torch.empty(B * L, device=kl_tok.device, dtype=torch.float32) if want_w else None
    call("fddm_kl_reduce", ptr(kl_tok), ptr(mask_u8), ptr(w), ptr(loss), B, L, stream())
    return loss, w


JUMP_FAST, JUMP_SAMPLE = 1, 2


def jump(logits2d, xt, coef, L, mode=0, temperature=1.0, seed=0, rng_stream=0, x_next=None, x0hat=None):
    """One jumpy-sampler step over logits [N, V] (f32): returns (x_next [N], x0hat [N]) int64."""
    N, V = logits2d.shape
    _chk(logits2d.dtype == torch.float32 and logits2d.stride(1) == 1, "jump: f32 rows with unit stride")
    _chk(xt.numel() == N and xt.dtype == torch.int64 and coef.dtype == torch.float32, "jump: xt/coef")
    _chk(coef.numel() >= 4 * ((N + L - 1) // L), "jump: coef holds 4 floats per batch element")
    if x_next is None:
        x_next = torch.empty(N, device=logits2d.device, dtype=torch.int64)
    if x0hat is None:
        x0hat = torch.empty(N, device=logits2d.device, dtype=torch.int64)
    call("fddm_jump", ptr(logits2d), logits2d.stride(0), ptr(xt), ptr(coef), ptr(x_next), ptr(x0hat), N, L, V, mode,
         float(temperature), seed, rng_stream, stream())
    return x_next, x0hat
