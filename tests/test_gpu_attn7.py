"""GPU parity of the 32x32x16-MFMA decoder attention kernels (csrc/attn7.hip) against float64 references with the
oracle's dropout mask (contract v2), at the shapes the decoder runs (keep bits written ahead by
fddm_attn_drop_bits, as models/denoise_decoder.py does) and at ragged / masked / extreme-score edge cases.

Tolerance: bf16 inputs and outputs, fp32 softmax statistics -> 2e-2 of the reference's max magnitude (tests/
test_gpu_kernels.py TOL for bf16); the LSE within LSE_ATOL absolute (natural-log units) where the row is finite.
fwd7 multiplies Q by scale*log2(e) once and rounds that to bf16 (one rounding of 2^-9 relative per element instead
of rounding the scores), so a score of magnitude |s| carries up to ~|s|*2^-9 of extra error; over randn inputs at
d=64 the LSE moves by up to ~2e-3, hence 4e-3 (the outputs stay within the bf16 2e-2 bar).
Reference: models/denoise_decoder.py:129-130,164,169-176 (nn.MultiheadAttention, key_padding_mask, dropout on
the probabilities).
"""
import pytest
import torch

from helpers import close
from oracle import fddm_oracle as O

pytestmark = pytest.mark.gpu
LSE_ATOL = 4e-3

dev = torch.device("cuda:0")
bf = torch.bfloat16


def ops():
    from fddm_hip import ops as o
    return o


def _ref(q, k, v, keep, p, seed, stream):
    """q [B,H,Lq,64] float64 ... -> O [B,H,Lq,64], lse [B,H,Lq] (natural log, of the scaled scores)."""
    B, H, Lq, _ = q.shape
    Lk = k.shape[2]
    s = (q @ k.transpose(-1, -2)) / 8.0
    if keep is not None:
        s = s.masked_fill(~keep[:, None, None, :], float("-inf"))
    lse = torch.logsumexp(s, -1)
    pr = torch.softmax(s, -1)
    if p > 0:
        m = O.attn_dropout_keep(seed, stream, B, H, Lq, Lk, p).double()
        pr = pr * m / (1 - p)
    return pr @ v, lse


def _run(B, H, Lq, Lk, keep, p, q, k, v, do=None, seed=5, stream=9, family="auto"):
    o = ops()
    D = H * 64
    to = lambda x: x.to(dev, bf).reshape(-1, D).contiguous()  # noqa: E731
    qd, kd, vd = to(q), to(k), to(v)
    od = torch.empty(B * Lq, D, device=dev, dtype=bf)
    lse = torch.empty(B * H, Lq, device=dev)
    kk = keep.to(dev).to(torch.uint8) if keep is not None else None
    db = None
    old = o.attn_force_kernels(family)    # the producer writes the selected family's storage layout
    try:
        if p > 0:
            db = o.drop_bits(B, H, Lq, Lk, dev).view(1, -1)
            o.attn_drop_bits(db, 1, B, H, Lq, Lk, p, seed, stream, 0)
            db = db.view(-1)
        o.attn_fwd(qd, kd, vd, od, lse, B, H, Lq, Lk, key_keep=kk, drop_p=p, seed=seed, rng_stream=stream, dbits=db,
                   bits_ready=db is not None)
        grads = None
        if do is not None:
            dq, dk, dv = torch.empty_like(qd), torch.empty_like(kd), torch.empty_like(vd)
            o.attn_bwd(qd, kd, vd, od, to(do), lse, dq, dk, dv, B, H, Lq, Lk, key_keep=kk, drop_p=p, seed=seed,
                       rng_stream=stream, dbits=db)
            grads = (dq, dk, dv)
    finally:
        o.attn_force_kernels(old)
    torch.cuda.synchronize()
    return od, lse, grads


def _heads(x, B, H):
    return x.to(bf).double().view(B, -1, H, 64).transpose(1, 2)


def _back(t):
    B, H, L, _ = t.shape
    return t.transpose(1, 2).reshape(B * L, H * 64)


SHAPES = [  # (B, H, Lq, Lk, key-padding mask, dropout p)
    (2, 3, 256, 256, True, 0.1),     # decoder self-attention (C2 geometry per head)
    (2, 3, 256, 499, False, 0.1),    # cross-attention, 10 s of audio (ragged last key tile)
    (2, 2, 512, 512, True, 0.1),     # C4 self
    (2, 2, 512, 499, False, 0.1),    # C4 cross
    (2, 3, 130, 70, True, 0.0),      # ragged queries and keys, no dropout
    (1, 2, 40, 1000, False, 0.1),    # long key range, a partial query block
    (2, 3, 129, 257, True, 0.1),
    (3, 1, 64, 64, False, 0.0),
    (2, 2, 200, 200, True, 0.1),
    (1, 1, 1, 1, False, 0.1),        # one query, one key
    (2, 2, 33, 5, True, 0.1),        # a partial 32-query group, five keys
    (1, 2, 96, 1024, True, 0.1),     # the longest key range of the 32x32x16 family (16 tiles, mask on every one)
    (1, 2, 96, 1025, False, 0.1),    # one key past it: the round-4 family takes the launch
]


@pytest.mark.parametrize("B,H,Lq,Lk,masked,p", SHAPES)
def test_attn7_forward_matches_float64(B, H, Lq, Lk, masked, p):
    D = H * 64
    gen = torch.Generator().manual_seed(Lq * 1000 + Lk)
    q, k, v = (torch.randn(B, L, D, generator=gen) for L in (Lq, Lk, Lk))
    keep = None
    if masked:
        keep = torch.ones(B, Lk, dtype=torch.bool)
        keep[B - 1, max(1, Lk - 9):] = False
        if Lk > 3:
            keep[0, 3] = False
        if Lk > 130:
            keep[B - 1, 64:128] = False  # a whole 64-key tile of padding inside the range (skipped tile)
    od, lse, _ = _run(B, H, Lq, Lk, keep, p, q, k, v)
    ref, rlse = _ref(_heads(q, B, H), _heads(k, B, H), _heads(v, B, H), keep, p, 5, 9)
    close(od.float(), _back(ref), rtol=2e-2, what="attn7 out")
    # with few keys the LSE is close to one score, whose error is the bf16 rounding of Q' (|s| 2^-9), not averaged
    smax = (_heads(q, B, H) @ _heads(k, B, H).transpose(-1, -2)).abs().max().item() / 8.0
    close(lse.view(B, H, Lq), rlse, rtol=0, atol=max(LSE_ATOL, 2.0 ** -8 * smax), what="attn7 lse")


@pytest.mark.parametrize("B,H,Lq,Lk,masked,p", [SHAPES[0], SHAPES[1], SHAPES[4], SHAPES[6], SHAPES[9], SHAPES[10],
                                                SHAPES[11], SHAPES[12]])
def test_attn7_forward_then_backward_matches_float64(B, H, Lq, Lk, masked, p):
    """The backward kernels read the forward's LSE and the same keep words: gradients vs float64 autograd."""
    D = H * 64
    gen = torch.Generator().manual_seed(7 + Lq + Lk)
    q, k, v, do = (torch.randn(B, L, D, generator=gen) for L in (Lq, Lk, Lk, Lq))
    keep = None
    if masked:
        keep = torch.ones(B, Lk, dtype=torch.bool)
        keep[B - 1, max(1, Lk - 9):] = False
    od, lse, (dq, dk, dv) = _run(B, H, Lq, Lk, keep, p, q, k, v, do)
    qr, kr, vr = (_heads(x, B, H).requires_grad_(True) for x in (q, k, v))
    ref, _ = _ref(qr, kr, vr, keep, p, 5, 9)
    ref.backward(_heads(do, B, H))
    close(od.float(), _back(ref.detach()), rtol=2e-2, what="out")
    # delta = rowsum(dO O) comes from the stored bf16 O: dS carries ~2^-9 |dO| |O| absolute error even where the
    # exact gradient vanishes (one key: softmax = 1, dQ = dK = 0 exactly), hence an absolute floor of 1e-2
    close(dq.float(), _back(qr.grad), rtol=6e-2, atol=1e-2, what="dq")
    close(dk.float(), _back(kr.grad), rtol=6e-2, atol=1e-2, what="dk")
    close(dv.float(), _back(vr.grad), rtol=6e-2, atol=1e-2, what="dv")


@pytest.mark.parametrize("B,H,Lq,Lk,masked,p", [(2, 3, 256, 256, True, 0.1), (2, 2, 300, 200, True, 0.1),
                                                (1, 2, 1, 256, False, 0.0), (2, 1, 65, 17, True, 0.1),
                                                (1, 1, 200, 240, False, 0.1), (2, 3, 256, 499, False, 0.1),
                                                (2, 2, 100, 300, True, 0.1), (1, 2, 256, 512, True, 0.0),
                                                (2, 1, 64, 257, False, 0.1), (2, 2, 200, 512, True, 0.1),
                                                (2, 2, 300, 400, True, 0.1)])  # the last: Lq > 256 -> the pair
def test_attn7_fused_backward_matches_float64_and_split_pair(B, H, Lq, Lk, masked, p):
    """Lk <= 256, or Lq <= 256 and Lk <= 512 (two key passes, the dQ partial kept in the workspace between them): the
    fused backward (bwdf7, one launch per (b, h) computing P and dP once, dQ from the dS^T image in LDS; the default)
    against float64 autograd, and against the split pair (dq7 + dkv7, family "nofused") on the same forward — two
    bf16 roundings of one float64 result (P, dS rounded to bf16 in both, sums in other orders)."""
    D = H * 64
    gen = torch.Generator().manual_seed(17 + Lq + Lk)
    q, k, v, do = (torch.randn(B, L, D, generator=gen) for L in (Lq, Lk, Lk, Lq))
    keep = None
    if masked:
        keep = torch.ones(B, Lk, dtype=torch.bool)
        keep[B - 1, max(1, Lk - 9):] = False
        if Lk > 130:
            keep[0, 64:128] = False  # a padded 64-key tile inside the range: two waves with no valid key
    _, _, gf = _run(B, H, Lq, Lk, keep, p, q, k, v, do, family="auto")
    _, _, gs = _run(B, H, Lq, Lk, keep, p, q, k, v, do, family="nofused")
    qr, kr, vr = (_heads(x, B, H).requires_grad_(True) for x in (q, k, v))
    ref, _ = _ref(qr, kr, vr, keep, p, 5, 9)
    ref.backward(_heads(do, B, H))
    for n, a_, b_, r in zip(("dq", "dk", "dv"), gf, gs, (qr.grad, kr.grad, vr.grad)):
        close(a_.float(), _back(r), rtol=6e-2, atol=1e-2, what=f"fused {n}")
        close(a_.float(), b_.float(), rtol=2e-2, atol=1e-2, what=f"fused vs split {n}")


@pytest.mark.parametrize("Lk", [256, 499])
def test_attn7_rescale_path_with_growing_scores(Lk):
    """Scores that grow along the keys (every 32-key half-tile exceeds the running maximum by far more than the
    2^8 rescale threshold) exercise the slow path on every half-tile; scores that fall along the keys keep the first
    half's reference. Forward against float64. The gradients at these scores (up to ~100, |K| up to ~25 per element)
    are bf16-limited in any kernel (dQ = scale sum_k dS K amplifies the bf16 rounding of P and dS by |K|): measured
    ~0.2-0.36 of max|dQ| for both families, so the backward is held to the round-4 family's error on the same inputs
    (within 1.5x) instead of to float64."""
    B, H, Lq = 2, 2, 128
    D = H * 64
    gen = torch.Generator().manual_seed(11)
    u = torch.randn(64, generator=gen)
    u = u / u.norm()
    q = (u * 4.0).repeat(B, Lq, H) + 0.05 * torch.randn(B, Lq, D, generator=gen)
    ramp = torch.linspace(0.0, 200.0, Lk)   # +6 to +13 scaled score units per 32-key half-tile
    for sign in (1.0, -1.0):
        k = (sign * ramp[None, :, None] * u.repeat(H)[None, None, :]).expand(B, Lk, D).contiguous()
        k = k + 0.05 * torch.randn(B, Lk, D, generator=gen)
        v = torch.randn(B, Lk, D, generator=gen)
        do = torch.randn(B, Lq, D, generator=gen)
        qr, kr, vr = (_heads(x, B, H).requires_grad_(True) for x in (q, k, v))
        ref, rlse = _ref(qr, kr, vr, None, 0.1, 5, 9)
        ref.backward(_heads(do, B, H))
        rg = [_back(x.grad) for x in (qr, kr, vr)]
        err = {}
        for fam in ("auto", "v6"):
            od, lse, grads = _run(B, H, Lq, Lk, None, 0.1, q, k, v, do, family=fam)
            if fam == "auto":
                close(od.float(), _back(ref.detach()), rtol=2e-2, what=f"out (sign {sign})")
                # the bf16 rounding of the pre-scaled Q moves scores by up to ~|s| 2^-9, as a bf16 rounding of the
                # scores themselves would (torch's bf16 bmm): a tolerance relative to the LSE
                close(lse.view(B, H, Lq), rlse.detach(), rtol=2.0 ** -9, atol=LSE_ATOL, what=f"lse (sign {sign})")
            err[fam] = [(g.float().cpu().double() - r).abs().max().item() / r.abs().max().item()
                        for g, r in zip(grads, rg)]
        for n, a_, b_ in zip(("dq", "dk", "dv"), err["auto"], err["v6"]):
            assert a_ <= 1.5 * b_ + 2e-2, f"{n} (sign {sign}): attn7 rel err {a_:.3g} vs round-4 family {b_:.3g}"


def test_attn7_fully_masked_rows_give_nan_like_softmax():
    """A batch whose keys are all padding: softmax over all -inf is NaN in the reference (torch), and so is every
    output and LSE of that batch here; the other batch is unaffected."""
    B, H, Lq, Lk = 2, 2, 96, 140
    D = H * 64
    gen = torch.Generator().manual_seed(3)
    q, k, v = (torch.randn(B, L, D, generator=gen) for L in (Lq, Lk, Lk))
    keep = torch.ones(B, Lk, dtype=torch.bool)
    keep[1] = False
    od, lse, _ = _run(B, H, Lq, Lk, keep, 0.1, q, k, v)
    o = od.float().view(B, Lq, D)
    assert torch.isnan(o[1]).all() and torch.isnan(lse.view(B, H, Lq)[1]).all()
    ref, _ = _ref(_heads(q, B, H), _heads(k, B, H), _heads(v, B, H), keep, 0.1, 5, 9)
    close(o[0], _back(ref)[: Lq].view(Lq, D), rtol=2e-2, what="unmasked batch")


@pytest.mark.parametrize("B,H,Lq,Lk,masked,p", [SHAPES[0], SHAPES[2], SHAPES[5]])
def test_attn7_agrees_with_round4_kernel(B, H, Lq, Lk, masked, p):
    """The 32x32x16 forward and the round-4 16x16x32 forward (fwd6, keep words read the same way) on the same
    inputs: both bf16 roundings of one float64 result, so within twice the per-kernel tolerance of each other."""
    D = H * 64
    gen = torch.Generator().manual_seed(99)
    q, k, v = (torch.randn(B, L, D, generator=gen) for L in (Lq, Lk, Lk))
    keep = None
    if masked:
        keep = torch.ones(B, Lk, dtype=torch.bool)
        keep[0, Lk - 30:] = False
    o7, l7, _ = _run(B, H, Lq, Lk, keep, p, q, k, v, family="auto")
    o6, l6, _ = _run(B, H, Lq, Lk, keep, p, q, k, v, family="v6")
    close(o7.float(), o6.float(), rtol=2e-2, what="fwd7 vs fwd6")
    close(l7, l6, rtol=0, atol=LSE_ATOL, what="lse fwd7 vs fwd6")


def test_attn7_forward_records_bits_when_not_ready():
    """attn_fwd with a keep-bit buffer that the producer has not filled (a standalone call, not the decoder's path):
    the 32x32x16 family writes the site's masks itself first, and the backward reads them."""
    o = ops()
    B, H, Lq, Lk, p = 2, 2, 96, 140, 0.1
    D = H * 64
    gen = torch.Generator().manual_seed(5)
    q, k, v, do = (torch.randn(B, L, D, generator=gen) for L in (Lq, Lk, Lk, Lq))
    to = lambda x: x.to(dev, bf).reshape(-1, D).contiguous()  # noqa: E731
    od = torch.empty(B * Lq, D, device=dev, dtype=bf)
    lse = torch.empty(B * H, Lq, device=dev)
    db = o.drop_bits(B, H, Lq, Lk, dev)
    o.attn_fwd(to(q), to(k), to(v), od, lse, B, H, Lq, Lk, drop_p=p, seed=5, rng_stream=9, dbits=db)
    dq, dk, dv = (torch.empty(B * L, D, device=dev, dtype=bf) for L in (Lq, Lk, Lk))
    o.attn_bwd(to(q), to(k), to(v), od, to(do), lse, dq, dk, dv, B, H, Lq, Lk, drop_p=p, seed=5, rng_stream=9,
               dbits=db)
    torch.cuda.synchronize()
    qr, kr, vr = (_heads(x, B, H).requires_grad_(True) for x in (q, k, v))
    ref, _ = _ref(qr, kr, vr, None, p, 5, 9)
    ref.backward(_heads(do, B, H))
    close(od.float(), _back(ref.detach()), rtol=2e-2, what="out")
    close(dk.float(), _back(kr.grad), rtol=6e-2, what="dk")


def test_decoder_long_audio_families_agree():
    """The whole bf16 decoder (training mode, dropout 0.1, keep bits written ahead by the producer for every block's
    two attention sites) with a condition longer than the 32x32x16 family takes (S = 1100 frames: the cross sites run
    on the round-4 kernels and read the round-4 words, the self sites on attn7 with layout v3): logits and every
    parameter gradient agree with the all-round-4 run on the same inputs and seeds (bf16 roundings of one result)."""
    from fddm_hip import runtime as rt
    from test_gpu_models import make_decoder
    o = ops()
    B, L, S, V, d, H, NL, FF = 2, 64, 1100, 300, 128, 2, 2, 256
    gen = torch.Generator().manual_seed(41)
    xt = torch.randint(1, V, (B, L), generator=gen)
    xt[1, 50:] = 0
    t = torch.tensor([3, 17])
    cond = torch.randn(B, S, d, generator=gen)
    R = torch.randn(B, L, V, generator=gen)
    res = {}
    for fam in ("auto", "v6"):
        old = o.attn_force_kernels(fam)
        try:
            with rt.use_precision("bf16"):
                torch.manual_seed(3)
                dec = make_decoder(V, d, H, NL, FF, dropout=0.1)
                dec.train()
                rt.reseed(11)
                logits = dec(xt.to(dev), t.to(dev), cond.to(dev), x_mask=(xt != 0).to(dev))
                (logits.float() * R.to(dev)).sum().backward()
                torch.cuda.synchronize()
                res[fam] = (logits.float().cpu(), {n: p.grad.float().cpu() for n, p in dec.named_parameters()
                                                   if p.grad is not None})
        finally:
            o.attn_force_kernels(old)
    close(res["auto"][0], res["v6"][0], rtol=3e-2, what="logits auto vs round-4")
    assert res["auto"][1].keys() == res["v6"][1].keys()
    for n in res["auto"][1]:
        close(res["auto"][1][n], res["v6"][1][n], rtol=6e-2, atol=1e-3, what=f"grad {n}")


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attn7_first_half_tile_masked_with_very_negative_scores(p):
    """a query whose first 32 keys are all padding keeps m = -inf after its first half-tile; with every
    valid score far below the running reference (here ~ -130 in log2 units) the fast path's exponentials underflow
    to 0 and the row sum stays 0 unless the slow path runs while no finite reference exists. Output and LSE must be
    finite and match float64 (torch's softmax is finite there)."""
    B, H, Lq, Lk = 1, 2, 64, 160
    D = H * 64
    gen = torch.Generator().manual_seed(13)
    u = torch.randn(64, generator=gen)
    u = u / u.norm()
    q = (u * 30.0).repeat(B, Lq, H) + 0.05 * torch.randn(B, Lq, D, generator=gen)
    k = (-u * 30.0).repeat(B, Lk, H) + 0.05 * torch.randn(B, Lk, D, generator=gen)   # q.k / 8 ~ -112
    v = torch.randn(B, Lk, D, generator=gen)
    keep = torch.ones(B, Lk, dtype=torch.bool)
    keep[:, :32] = False
    od, lse, _ = _run(B, H, Lq, Lk, keep, p, q, k, v)
    assert torch.isfinite(od.float()).all() and torch.isfinite(lse).all()
    ref, rlse = _ref(_heads(q, B, H), _heads(k, B, H), _heads(v, B, H), keep, p, 5, 9)
    close(od.float(), _back(ref), rtol=2e-2, what="out")
    close(lse.view(B, H, Lq), rlse, rtol=2.0 ** -8, atol=LSE_ATOL, what="lse")


@pytest.mark.parametrize("B,H,Lq,Lk,masked,p", [SHAPES[0], SHAPES[1], SHAPES[2], SHAPES[4], SHAPES[6], SHAPES[9],
                                                SHAPES[10], SHAPES[11], (2, 2, 600, 300, True, 0.1)])
def test_fwd8_agrees_with_fwd7(B, H, Lq, Lk, masked, p):
    """The two-chain forward (attn8.hip fwd8, forced; the default where its grid loads no CU more than fwd7's) against
    the one-chain fwd7 on the same inputs and keep bits:
    same score operands (pre-scaled Q'), different reference handling (fwd8 fixes each chain's reference at its first
    half-tile), so both are bf16 roundings of one float64 result."""
    D = H * 64
    gen = torch.Generator().manual_seed(123 + Lq + Lk)
    q, k, v = (torch.randn(B, L, D, generator=gen) for L in (Lq, Lk, Lk))
    keep = None
    if masked:
        keep = torch.ones(B, Lk, dtype=torch.bool)
        keep[B - 1, max(1, Lk - 9):] = False
        if Lk > 130:
            keep[0, 64:128] = False
    o8, l8, _ = _run(B, H, Lq, Lk, keep, p, q, k, v, family="fwd8")
    o7, l7, _ = _run(B, H, Lq, Lk, keep, p, q, k, v, family="fwd7")
    close(o8.float(), o7.float(), rtol=2e-2, what="fwd8 vs fwd7")
    close(l8, l7, rtol=0, atol=LSE_ATOL, what="lse fwd8 vs fwd7")
