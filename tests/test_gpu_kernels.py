"""GPU parity tests of each libfddm_hip kernel against the CPU oracle / float64 references.

Tolerances: fp32 kernels (exact f32 MFMA) within 1e-4 relative of the max reference magnitude
(the north-star bar for fp32 logits/loss); bf16 kernels within 2e-2 relative; integer outputs
(sampled token ids, dropout masks) bit-exact.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import close
from oracle import fddm_oracle as O

pytestmark = pytest.mark.gpu

dev = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    import fddm_hip  # noqa: F401  (loads libfddm_hip.so, raises if absent)
    from fddm_hip import ops
    assert torch.cuda.is_available()
    return ops


@pytest.fixture
def gemm_path():
    """Setter of the GEMM kernel-family override (ops.gemm_force_path); restores the automatic choice afterwards."""
    from fddm_hip import ops as o
    yield o.gemm_force_path
    o.gemm_force_path("auto")


def ops():
    from fddm_hip import ops as o
    return o


TOL = {torch.float32: 1e-4, torch.bfloat16: 2e-2}


def g(seed):
    return torch.Generator().manual_seed(seed)


# ------------------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("a_kc,b_kc", [(1, 1), (1, 0), (0, 0), (0, 1)])
@pytest.mark.parametrize("M,N,K", [(200, 136, 96), (128, 128, 256), (8, 264, 520)])
def test_gemm_layouts(dtype, a_kc, b_kc, M, N, K):
    o = ops()
    A = torch.randn(M, K, generator=g(1))
    Bm = torch.randn(N, K, generator=g(2))
    bias = torch.randn(N, generator=g(3))
    ref = A.double() @ Bm.double().T + bias.double()
    Ad = (A if a_kc else A.T.contiguous()).to(dev, dtype)
    Bd = (Bm if b_kc else Bm.T.contiguous()).to(dev, dtype)
    C = torch.zeros(M, N, device=dev, dtype=torch.float32)
    o.gemm(Ad, Bd, C, M, N, K, a_kc=bool(a_kc), b_kc=bool(b_kc), lda=K if a_kc else M, ldb=K if b_kc else N, ldc=N,
           bias=bias.to(dev))
    torch.cuda.synchronize()
    if dtype == torch.bfloat16:
        ref = A.bfloat16().double() @ Bm.bfloat16().double().T + bias.double()
    close(C, ref, rtol=1e-5 if dtype == torch.float32 else 1e-3, what="gemm")


def test_gemm_epilogues_and_mixed_a():
    o = ops()
    M, N, K = 192, 160, 128
    A = torch.randn(M, K, generator=g(4))
    W = torch.randn(N, K, generator=g(5)) / math.sqrt(K)
    b = torch.randn(N, generator=g(6))
    Ad, Wd, bd = A.to(dev).bfloat16(), W.to(dev).bfloat16(), b.to(dev)
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    act = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    o.linear(Ad, Wd, bd, out=pre, epi=o.EPI_GELU, C2=act, drop_p=0.1, seed=7, rng_stream=3)
    ref = A.bfloat16().double() @ W.bfloat16().double().T + b.double()
    keep = O.dropout_keep(7, 3, M * N, 0.1).view(M, N)
    close(pre.float(), ref, rtol=1e-2, what="gelu pre")
    close(act.float(), F.gelu(ref) * keep / 0.9, rtol=2e-2, what="gelu act+dropout")
    # mixed: A stored f32, bf16 compute; accumulate epilogue
    C = torch.ones(M, N, device=dev)
    o.gemm(A.to(dev), Wd, C, M, N, K, lda=K, ldb=K, ldc=N, epi=o.EPI_ACC)
    close(C, 1 + A.bfloat16().double() @ W.bfloat16().double().T, rtol=1e-2, what="mixed acc")
    # dGELU epilogue
    dy = torch.randn(M, K, generator=g(8))
    dh = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    Wt = torch.randn(K, N, generator=g(9))  # [N_out=K][in=N] weight -> dx = dy @ Wt
    o.linear_dx(dy.to(dev).bfloat16(), Wt.to(dev).bfloat16(), out=dh, epi=o.EPI_DGELU, C2=pre, drop_p=0.1, seed=7,
                rng_stream=3)
    x = pre.float().cpu().double()
    cdf = 0.5 * (1 + torch.erf(x / math.sqrt(2)))
    gg = cdf + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)
    refd = (dy.bfloat16().double() @ Wt.bfloat16().double()) * gg * keep / 0.9
    close(dh.float(), refd, rtol=2e-2, what="dgelu")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(200, 136, 96), (512, 256, 8192), (24, 512, 300)])
def test_weight_grad_gemm_with_fused_bias_grad(dtype, M, N, K):
    """dW = dy^T x (split-K when the output has few tiles) and db = colsum(dy) in the same launch."""
    o = ops()
    dy = torch.randn(K, M, generator=g(15))
    x = torch.randn(K, N, generator=g(16))
    dW = torch.empty(M, N, device=dev)
    db = torch.empty(M, device=dev)
    o.linear_dw(dy.to(dev, dtype), x.to(dev, dtype), out=dW, db=db)
    ref = dy.to(dtype).double().T @ x.to(dtype).double()
    close(dW, ref, rtol=1e-5 if dtype == torch.float32 else 1e-3, what="dW")
    close(db, dy.to(dtype).double().sum(0), rtol=1e-5 if dtype == torch.float32 else 1e-3, what="db")


@pytest.mark.parametrize("path", ["256", "big", "128"])
@pytest.mark.parametrize("M,N,K,epi,odt", [(8192, 2048, 512, 0, "bf16"), (15968, 768, 3072, 1, "bf16"),
                                           (8200, 2056, 768, 3, "bf16"), (8192, 8000, 512, 0, "f32"),
                                           (300, 264, 64, 0, "bf16"), (1000, 3072, 192, 1, "bf16")])
def test_big_gemm_matches_torch(M, N, K, epi, odt, path, monkeypatch, gemm_path):
    """256x256 8-phase GEMM / 256x128 LDS-DMA GEMM (ops.gemm_force_path) vs torch fp32 on the same bf16 operands,
    and vs the 128x128 path — ragged M/N edges, f32 output, dropout-free GELU epilogues included."""
    o = ops()
    gen = torch.Generator(device=dev).manual_seed(3)
    A = torch.randn(M, K, device=dev, generator=gen).bfloat16()
    W = (torch.randn(N, K, device=dev, generator=gen) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev, generator=gen)
    ref = A.float() @ W.float().T + b
    odtype = torch.float32 if odt == "f32" else torch.bfloat16
    out = torch.full((M, N), float("nan"), device=dev, dtype=odtype)
    act = torch.full((M, N), float("nan"), device=dev, dtype=odtype)
    gemm_path(path)
    o.gemm(A, W, out, M, N, K, lda=K, ldb=K, ldc=N, bias=b, epi=epi, C2=act if epi == 1 else None)
    chk = (act if epi == 1 else out).float()
    want = F.gelu(ref) if epi in (1, 3) else ref
    err = (chk - want).abs().max().item()
    assert err <= 2e-2 * want.abs().max().item(), err
    if epi == 1:
        assert (out.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    gemm_path("small")
    out2 = torch.empty_like(out)
    act2 = torch.empty_like(act)
    o.gemm(A, W, out2, M, N, K, lda=K, ldb=K, ldc=N, bias=b, epi=epi, C2=act2 if epi == 1 else None)
    chk2 = (act2 if epi == 1 else out2).float()
    assert (chk - chk2).abs().max().item() <= 1e-2 * want.abs().max().item()


def test_grouped_weight_grads_match_torch():
    """fddm_gemm_dw_grouped: the dW / db GEMMs of a decoder block in one launch (ragged K split across
    workgroups, strided column slices of one gradient buffer) accumulate like torch in fp64."""
    o = ops()
    gen = torch.Generator(device=dev).manual_seed(11)
    Kt, Kc = 1000, 1996
    shapes = [(Kt, 64, 256), (Kt, 256, 64), (Kc, 128, 64), (Kt, 64, 64)]
    dW = torch.randn(256 + 64 + 64, 256, device=dev, generator=gen)  # row slices for several jobs
    dW0 = dW.clone()
    db = torch.randn(512, device=dev, generator=gen)
    db0 = db.clone()
    jobs, refs = [], []
    r0 = 0
    for i, (K, M, N) in enumerate(shapes):
        dy = torch.randn(K, M, device=dev, generator=gen).bfloat16()
        x = torch.randn(K, N, device=dev, generator=gen).bfloat16()
        if i == 0:
            dst, bdst = dW[r0:r0 + M, :N], db[:M]
        elif i == 1:
            dst, bdst = torch.zeros(M, N, device=dev), None
        elif i == 2:
            dst, bdst = dW[r0:r0 + M, :N], db[256:256 + M]
        else:
            dst, bdst = dW[r0:r0 + M, 64:64 + N], db[448:448 + M]
        jobs.append((dy, x, dst, bdst))
        refs.append((dy.double().T @ x.double(), dy.double().sum(0)))
        if i != 1:
            r0 += M
    o.linear_dw_grouped(jobs, kchunk=512)
    close(jobs[1][2], refs[1][0], rtol=1e-4, what="dW job1")
    close(dW[0:64, :256], dW0[0:64, :256].double() + refs[0][0], rtol=1e-4, what="dW job0")
    close(dW[64:192, :64], dW0[64:192, :64].double() + refs[2][0], rtol=1e-4, what="dW job2")
    close(dW[192:256, 64:128], dW0[192:256, 64:128].double() + refs[3][0], rtol=1e-4, what="dW job3")
    close(db[:64], db0[:64].double() + refs[0][1], rtol=1e-4, what="db0")
    close(db[256:384], db0[256:384].double() + refs[2][1], rtol=1e-4, what="db2")


@pytest.mark.parametrize("M,N,K", [(1000, 520, 512), (8192, 512, 2048), (128, 128, 64), (4100, 1000, 320),
                                   (8192, 2048, 512)])
def test_gemm128_input_grad_layout(M, N, K, monkeypatch, gemm_path):
    """128x128 LDS-DMA kernel, A K-contiguous x B as stored [K][N] (dX = dY W): f32 store / accumulate,
    bf16 store, dGELU+dropout epilogue — against torch in fp64 on the same bf16 operands."""
    o = ops()
    gemm_path("128")
    gen = torch.Generator(device=dev).manual_seed(21)
    dy = torch.randn(M, K, device=dev, generator=gen).bfloat16()
    W = (torch.randn(K, N, device=dev, generator=gen) / math.sqrt(K)).bfloat16()
    ref = dy.double() @ W.double()
    out = torch.full((M, N), float("nan"), device=dev)
    o.linear_dx(dy, W, out=out)
    close(out, ref, rtol=1e-4, what="dx f32")
    base = torch.randn(M, N, device=dev, generator=gen)
    acc = base.clone()
    o.linear_dx(dy, W, out=acc, accumulate=True)
    close(acc, base.double() + ref, rtol=1e-4, what="dx acc")
    ob = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    o.linear_dx(dy, W, out=ob, out_dtype=torch.bfloat16)
    close(ob.float(), ref, rtol=1e-2, what="dx bf16")
    pre = torch.randn(M, N, device=dev, generator=gen).bfloat16()
    dh = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    o.linear_dx(dy, W, out=dh, epi=o.EPI_DGELU, C2=pre, drop_p=0.1, seed=9, rng_stream=4)
    x = pre.double()
    gg = 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)
    keep = O.dropout_keep(9, 4, M * N, 0.1).view(M, N).to(dev)
    close(dh.float(), ref * gg * keep / 0.9, rtol=2e-2, what="dgelu")
    gemm_path("small")
    dh2 = torch.empty_like(dh)
    o.linear_dx(dy, W, out=dh2, epi=o.EPI_DGELU, C2=pre, drop_p=0.1, seed=9, rng_stream=4)
    # the same dropped elements in both families (elements whose product rounds to zero in one of them aside:
    # at 8192 x 2048 one sum of 512 products comes out exactly 0 in one accumulation order, -2.8e-9 in the other)
    big = (ref.abs() > 1e-3).to(dev)
    assert torch.equal((dh == 0) & big, (dh2 == 0) & big)


def test_gemm128_repeats_and_graph_replay(monkeypatch, gemm_path):
    """A 4-round 128x128 launch (1024 tiles): back-to-back launches, accumulating launches, and a launch captured in
    a HIP graph and replayed beside eager ones all give bit-identical results (every tile computed exactly once, by
    the same arithmetic whichever workgroup takes it)."""
    o = ops()
    gemm_path("128")
    gen = torch.Generator(device=dev).manual_seed(31)
    M, N, K = 8192, 2048, 512
    dy = torch.randn(M, K, device=dev, generator=gen).bfloat16()
    W = (torch.randn(K, N, device=dev, generator=gen) / math.sqrt(K)).bfloat16()
    ref = torch.empty(M, N, device=dev)
    o.linear_dx(dy, W, out=ref)
    close(ref, dy.double() @ W.double(), rtol=1e-4, what="dx")
    for _ in range(5):
        out = torch.full((M, N), float("nan"), device=dev)
        o.linear_dx(dy, W, out=out)
        assert torch.equal(out, ref)
    acc = torch.zeros(M, N, device=dev)
    for _ in range(3):
        o.linear_dx(dy, W, out=acc, accumulate=True)
    close(acc, 3 * ref.double(), rtol=1e-5, what="3 accumulating launches")
    gout = torch.full((M, N), float("nan"), device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            o.linear_dx(dy, W, out=gout)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        gout.fill_(float("nan"))
        g.replay()
        eager = torch.full((M, N), float("nan"), device=dev)
        o.linear_dx(dy, W, out=eager)
        torch.cuda.synchronize()
        assert torch.equal(gout, ref) and torch.equal(eager, ref)


@pytest.mark.parametrize("M,N,K", [(264, 200, 1000), (512, 512, 8192), (128, 128, 4096), (1024, 512, 15968)])
def test_gemm128_weight_grad_layout(M, N, K, monkeypatch, gemm_path):
    """128x128 LDS-DMA kernel, both operands token-major (dW = dY^T X): ragged token counts read zeros past the
    end, split-K slices accumulate atomically, the bias gradient (colsum) is fused."""
    o = ops()
    gemm_path("128")
    gen = torch.Generator(device=dev).manual_seed(22)
    dy = torch.randn(K, M, device=dev, generator=gen).bfloat16()
    x = torch.randn(K, N, device=dev, generator=gen).bfloat16()
    ref = dy.double().T @ x.double()
    dW = torch.full((M, N), float("nan"), device=dev)
    db = torch.full((M,), float("nan"), device=dev)
    o.linear_dw(dy, x, out=dW, db=db)
    close(dW, ref, rtol=1e-4, what="dW")
    close(db, dy.double().sum(0), rtol=1e-4, what="db")
    o.linear_dw(dy, x, out=dW, db=db, accumulate=True)
    close(dW, 2 * ref, rtol=1e-4, what="dW acc")
    close(db, 2 * dy.double().sum(0), rtol=1e-4, what="db acc")


def test_gemm128_grouped_weight_grads(monkeypatch, gemm_path):
    """The decoder block's 8 weight-gradient GEMMs in one 128x128 grouped launch (automatic split balance):
    token counts 8192 / 15968 (ragged), column slices of shared gradient buffers, fused bias gradients."""
    o = ops()
    gemm_path("auto")
    gen = torch.Generator(device=dev).manual_seed(23)
    T, d, FF, TS = 2048, 256, 1024, 3992
    specs = [(T, d, FF), (T, FF, d), (T, d, d), (T, d, d), (TS, 2 * d, d), (T, d, d), (T, 2 * d, d), (T, d, d)]
    jobs, refs = [], []
    for K, M, N in specs:
        dy = torch.randn(K, M, device=dev, generator=gen).bfloat16()
        x = torch.randn(K, N, device=dev, generator=gen).bfloat16()
        dW = torch.randn(M, N + 16, device=dev, generator=gen)[:, 8:8 + N]
        db = torch.randn(M, device=dev, generator=gen)
        refs.append((dW.double() + dy.double().T @ x.double(), db.double() + dy.double().sum(0)))
        jobs.append((dy, x, dW, db))
    o.linear_dw_grouped(jobs)
    for i, ((dy, x, dW, db), (rw, rb)) in enumerate(zip(jobs, refs)):
        close(dW, rw, rtol=1e-4, what=f"dW job{i}")
        close(db, rb, rtol=1e-4, what=f"db job{i}")


def test_grouped_weight_grads_ragged_tiles(monkeypatch, gemm_path):
    """Grouped weight gradients: ragged rows and columns (shifted last tiles, overlap added once), ragged token
    counts, a split-K problem among read-modify-write ones (the batched read-modify-write epilogue), strided
    destinations, fused bias gradients."""
    o = ops()
    gemm_path("auto")
    gen = torch.Generator(device=dev).manual_seed(29)
    specs = [(1000, 200, 320), (8192, 1536, 512), (3992, 136, 264), (15968, 256, 512), (2048, 384, 768)]
    jobs, refs = [], []
    for K, M, N in specs:
        dy = torch.randn(K, M, device=dev, generator=gen).bfloat16()
        x = torch.randn(K, N, device=dev, generator=gen).bfloat16()
        dW = torch.randn(M, N + 24, device=dev, generator=gen)[:, 8:8 + N]
        db = torch.randn(M, device=dev, generator=gen)
        refs.append((dW.double() + dy.double().T @ x.double(), db.double() + dy.double().sum(0)))
        jobs.append((dy, x, dW, db))
    o.linear_dw_grouped(jobs)
    for i, ((dy, x, dW, db), (rw, rb)) in enumerate(zip(jobs, refs)):
        close(dW, rw, rtol=1e-4, what=f"dW job{i}")
        close(db, rb, rtol=1e-4, what=f"db job{i}")


def test_gemm256_dropout_gelu_matches_small_path(monkeypatch, gemm_path):
    """EPI_GELU with dropout: the 256x256 epilogue draws the same keep mask (counter-based hash of m*N+n)."""
    o = ops()
    M, N, K, p = 1100, 2048, 512, 0.1
    gen = torch.Generator(device=dev).manual_seed(5)
    A = torch.randn(M, K, device=dev, generator=gen).bfloat16()
    W = (torch.randn(N, K, device=dev, generator=gen) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev, generator=gen)
    outs = []
    for path in ("256", "small"):
        gemm_path(path)
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        act = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        o.gemm(A, W, pre, M, N, K, lda=K, ldb=K, ldc=N, bias=b, epi=1, C2=act, drop_p=p, seed=7, rng_stream=3)
        outs.append((pre.float(), act.float()))
    assert torch.equal(outs[0][1] == 0, outs[1][1] == 0)
    assert (outs[0][1] - outs[1][1]).abs().max().item() <= 2e-2 * outs[1][1].abs().max().item()


@pytest.mark.parametrize("path", ["256", "big"])
def test_big_conv_gemm_matches_torch(path, monkeypatch, gemm_path):
    o = ops()
    B, Cin, Tin, Cout, k, s = 8, 512, 4001, 512, 3, 2
    gen = torch.Generator(device=dev).manual_seed(4)
    x = torch.randn(B, Tin, Cin, device=dev, generator=gen).bfloat16()
    w = (torch.randn(Cout, Cin, k, device=dev, generator=gen) / math.sqrt(Cin * k)).bfloat16()
    ref = F.gelu(F.conv1d(x.float().transpose(1, 2), w.float(), stride=s)).transpose(1, 2)
    Tout = ref.shape[1]
    Wp = w.permute(0, 2, 1).contiguous()
    out = torch.empty(B, Tout, Cout, device=dev, dtype=torch.bfloat16)
    gemm_path(path)
    o.conv1d_gemm(x, Wp, out, lda=Cin, sAb=Tin * Cin, Tin=Tin, Cg=Cin, cstride=s, cpad=0, Bn=B, Tout=Tout, N=Cout,
                  K=k * Cin, gelu=True)
    err = (out.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err


def test_gelu_fast_erf_accuracy():
    o = ops()
    x = torch.linspace(-8, 8, 4096).view(32, 128)
    W = torch.eye(128)
    pre = torch.empty(32, 128, device=dev)
    act = torch.empty(32, 128, device=dev)
    o.linear(x.to(dev), W.to(dev), None, out=pre, epi=o.EPI_GELU, C2=act)
    close(act, F.gelu(x.double()), rtol=0, atol=2e-6, what="gelu")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv1d_gemm_matches_conv(dtype):
    o = ops()
    B, Cin, Tin, Cout, k, s = 2, 64, 101, 64, 3, 2
    x = torch.randn(B, Cin, Tin, generator=g(10))
    w = torch.randn(Cout, Cin, k, generator=g(11)) / math.sqrt(Cin * k)
    ref = F.conv1d(x.double(), w.double(), stride=s)            # [B, Cout, Tout]
    Tout = ref.shape[-1]
    xd = x.transpose(1, 2).contiguous().to(dev, dtype)
    Wp = w.permute(0, 2, 1).contiguous().to(dev, dtype)
    out = torch.empty(B, Tout, Cout, device=dev, dtype=dtype)
    o.conv1d_gemm(xd, Wp, out, lda=Cin, sAb=Tin * Cin, Tin=Tin, Cg=Cin, cstride=s, cpad=0, Bn=B, Tout=Tout, N=Cout,
                  K=k * Cin, gelu=True)
    close(out.float().transpose(1, 2), F.gelu(ref), rtol=TOL[dtype], what="conv")
    # grouped, padded (positional conv geometry scaled down)
    E, G, kp, S = 64, 4, 16, 37
    Cg = E // G
    x = torch.randn(B, E, S, generator=g(12))
    w = torch.randn(E, Cg, kp, generator=g(13)) / math.sqrt(Cg * kp)
    bb = torch.randn(E, generator=g(14))
    ref = F.conv1d(x.double(), w.double(), bb.double(), padding=kp // 2, groups=G)[:, :, :-1]
    Wp = w.view(G, Cg, Cg, kp).permute(0, 1, 3, 2).contiguous().to(dev, dtype)
    out = torch.empty(B * S, E, device=dev, dtype=dtype)
    o.conv1d_gemm(x.transpose(1, 2).contiguous().to(dev, dtype), Wp, out, lda=E, sAb=S * E, Tin=S, Cg=Cg, cstride=1,
                  cpad=kp // 2, Bn=B, Tout=S, N=Cg, K=kp * Cg, groups=G, bias=bb.to(dev), gelu=True)
    close(out.float().view(B, S, E).transpose(1, 2), F.gelu(ref), rtol=TOL[dtype], what="grouped conv")


@pytest.mark.parametrize("S", [37, 499])
def test_posconv_matches_conv(S):
    """WavLM positional conv (kernel 128, pad 64, 16 -> here 4 groups of 48, SamePad, GELU) of the bf16
    whole-window kernel vs torch conv1d in fp64 on the same bf16 operands."""
    o = ops()
    B, E, G, kp = 3, 192, 4, 128
    Cg = E // G
    gen = torch.Generator().manual_seed(21)
    x = torch.randn(B, S, E, generator=gen).bfloat16()
    w = (torch.randn(E, Cg, kp, generator=gen) / math.sqrt(Cg * kp)).bfloat16()
    bb = torch.randn(E, generator=gen)
    ref = F.conv1d(x.double().transpose(1, 2), w.double(), bb.double(), padding=kp // 2, groups=G)[:, :, :-1]
    ref = F.gelu(ref).transpose(1, 2)
    Wp = w.view(G, Cg, Cg, kp).permute(0, 1, 3, 2).contiguous().to(dev)
    out = torch.full((B * S, E), float("nan"), device=dev, dtype=torch.bfloat16)
    o.posconv_gelu(x.to(dev).reshape(B * S, E).contiguous(), Wp, bb.to(dev), out, B, S, E, G, kp)
    close(out.float().view(B, S, E), ref, rtol=2e-2, what="posconv")


# ------------------------------------------------------------------------------------- attention
def _attn_ref(q, k, v, keep, p_drop, seed, stream, gate=None, table=None):
    """q [B,H,Lq,64] ... float64 reference with the oracle's dropout mask."""
    B, H, Lq, _ = q.shape
    Lk = k.shape[2]
    s = (q @ k.transpose(-1, -2)) / 8.0
    if table is not None:
        rel = torch.arange(Lk)[None, :] - torch.arange(Lq)[:, None] + Lk - 1
        s = s + gate[..., None] * table[:, rel][None]
    if keep is not None:
        s = s.masked_fill(~keep[:, None, None, :], float("-inf"))
    pr = torch.softmax(s, -1)
    if p_drop > 0:
        m = O.attn_dropout_keep(seed, stream, B, H, Lq, Lk, p_drop).double()
        pr = pr * m / (1 - p_drop)
    return pr @ v


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Lq,Lk,masked,p,bits", [(70, 70, True, 0.0, False), (64, 130, False, 0.1, False),
                                                 (33, 49, True, 0.1, False), (150, 200, True, 0.1, True),
                                                 (64, 130, False, 0.1, True), (40, 499, False, 0.1, True),
                                                 (129, 257, True, 0.1, True), (96, 256, True, 0.1, True),
                                                 (64, 499, False, 0.0, False), (256, 256, False, 0.1, True),
                                                 (200, 200, True, 0.1, True), (32, 32, False, 0.0, False),
                                                 (512, 512, True, 0.1, True), (300, 499, False, 0.1, True),
                                                 (40, 1100, True, 0.1, True), (1100, 70, False, 0.1, True)])
def test_attention_fwd_bwd(dtype, Lq, Lk, masked, p, bits):
    """bits: the forward records the dropout keep bits and the backward reads them (bf16 path). The shapes reach every
    bf16 kernel the dispatch (csrc/attention.hip run<T>) selects: fwd6 for Lk <= 1024 (keep bits drawn in-kernel and
    recorded, or rehashed later when no buffer is given), fwd2 past that; the fused bwd3s for Lq == Lk <= 256 with
    recorded bits; dq4 / dkv4 up to 1024; dq2 / dkv2 for rehashed bits or longer sequences (1100)."""
    o = ops()
    B, H = 2, 3
    D = H * 64
    q = torch.randn(B, Lq, D, generator=g(20))
    k = torch.randn(B, Lk, D, generator=g(21))
    v = torch.randn(B, Lk, D, generator=g(22))
    do = torch.randn(B, Lq, D, generator=g(23))
    keep = None
    if masked:
        keep = torch.ones(B, Lk, dtype=torch.bool)
        keep[1, Lk - 9:] = False
    to = lambda x: x.to(dev, dtype).reshape(-1, D).contiguous()  # noqa: E731
    qd, kd, vd, dod = to(q), to(k), to(v), to(do)
    od = torch.empty(B * Lq, D, device=dev, dtype=dtype)
    lse = torch.empty(B * H, Lq, device=dev)
    kk = keep.to(dev).to(torch.uint8) if keep is not None else None
    db = o.drop_bits(B, H, Lq, Lk, dev) if bits else None
    o.attn_fwd(qd, kd, vd, od, lse, B, H, Lq, Lk, key_keep=kk, drop_p=p, seed=5, rng_stream=9, dbits=db)
    dq = torch.empty_like(qd)
    dk = torch.empty_like(kd)
    dv = torch.empty_like(vd)
    o.attn_bwd(qd, kd, vd, od, dod, lse, dq, dk, dv, B, H, Lq, Lk, key_keep=kk, drop_p=p, seed=5, rng_stream=9,
               dbits=db)
    torch.cuda.synchronize()
    hv = lambda x: x.to(dtype).double().view(B, -1, H, 64).transpose(1, 2)  # noqa: E731
    qr, kr, vr = (hv(x).requires_grad_(True) for x in (q, k, v))
    ref = _attn_ref(qr, kr, vr, keep, p, 5, 9)
    ref.backward(hv(do))
    back = lambda t: t.transpose(1, 2).reshape(B * t.shape[2], D)  # noqa: E731
    tol = TOL[dtype]
    close(od.float(), back(ref.detach()), rtol=tol, what="attn out")
    close(dq.float(), back(qr.grad), rtol=3 * tol, what="dq")
    close(dk.float(), back(kr.grad), rtol=3 * tol, what="dk")
    close(dv.float(), back(vr.grad), rtol=3 * tol, what="dv")


def _decode_v3(w, BH, Lq, Lk):
    """Storage layout v3 (csrc/attn7.hip lane masks) -> keep [BH, Lq, Lk]: word ((bh*nqg + qg)*nt + t)*32 + 16kb + r,
    bit l = keep(query 32qg + (l&31), key 64t + 32kb + 8(r>>2) + 4(l>>5) + (r&3))."""
    nqg, nt = (Lq + 31) // 32, (Lk + 63) // 64
    bits = ((w.view(BH, nqg, nt, 2, 16, 1) >> torch.arange(64, dtype=torch.int64)) & 1).bool()  # [BH,nqg,nt,kb,r,l]
    r = torch.arange(16)[:, None]
    l = torch.arange(64)[None, :]
    q_of = (l & 31).expand(16, 64)                                  # query within the group
    k_of = (8 * (r >> 2) + 4 * (l >> 5) + (r & 3)).expand(16, 64)   # key within the 32-key half
    out = torch.zeros(BH, nqg * 32, nt * 64, dtype=torch.bool)
    for g in range(nqg):
        for t in range(nt):
            for kb in range(2):
                out[:, 32 * g + q_of, 64 * t + 32 * kb + k_of] = bits[:, g, t, kb]
    return out[:, :Lq, :Lk]


def _decode_v5(w, BH, Lq, Lk):
    """The per-lane dwords after the lane masks (layout v5, csrc/attn7_common.h lb_bit) -> keep [BH, Lq, Lk]: dword
    ((bh*nqg + qg)*nt + t)*64 + l, register r of half kb at bit 15 - p (r even) or 31 - p (r odd), p = 8kb + (r>>1);
    register r of lane l is query 32qg + (l&31), key 64t + 32kb + 8(r>>2) + 4(l>>5) + (r&3)."""
    nqg, nt = (Lq + 31) // 32, (Lk + 63) // 64
    d = (w & 0xFFFFFFFF).view(BH, nqg, nt, 64)
    out = torch.zeros(BH, nqg * 32, nt * 64, dtype=torch.bool)
    lanes = torch.arange(64)
    for kb in range(2):
        for r in range(16):
            p_ = 8 * kb + (r >> 1)
            bit = (31 if r & 1 else 15) - p_
            v = ((d >> bit) & 1).bool()                                     # [BH, nqg, nt, 64 lanes]
            key = 32 * kb + 8 * (r >> 2) + 4 * (lanes >> 5) + (r & 3)
            for g in range(nqg):
                for t in range(nt):
                    out[:, 32 * g + (lanes & 31), 64 * t + key] = v[:, g, t]
    return out[:, :Lq, :Lk]


@pytest.mark.parametrize("family", ["auto", "v6"])
@pytest.mark.parametrize("Lq,Lk", [(256, 256), (40, 499), (129, 70)])
def test_attention_drop_bits_producer_matches_oracle(Lq, Lk, family):
    """fddm_attn_drop_bits (the decoder writes every block's attention-dropout keep bits in two launches ahead of the
    forward): 3 sites of one shape, rng streams 7, 13, 19, against the oracle's contract-v2 mask bit for bit, in the
    storage layout the selected kernel family reads: layout v3 lane masks and the v5 per-lane dwords after them
    (default, csrc/attn7.hip, attn7_common.h) or the round-4
    words (bit kk of word (bh, t, q) = keep(q, key 64t + kk))."""
    o = ops()
    B, H, p, seed = 2, 3, 0.1, 77
    nt = (Lk + 63) // 64
    words = o.drop_words(B, H, Lq, Lk)
    out = torch.zeros(3, words + 5, device=dev, dtype=torch.int64)
    old = o.attn_force_kernels(family)
    try:
        o.attn_drop_bits(out, 3, B, H, Lq, Lk, p, seed, 7, 6)
    finally:
        o.attn_force_kernels(old)
    torch.cuda.synchronize()
    assert (out[:, words:] == 0).all(), "wrote past the site's words"
    bitpos = torch.arange(64, dtype=torch.int64)
    for s_ in range(3):
        if family == "v6":
            w = out[s_, :B * H * nt * Lq].cpu().view(B * H, nt, Lq)
            bits = ((w[..., None] >> bitpos) & 1).bool()                       # [BH, nt, Lq, 64]
            got = bits.permute(0, 2, 1, 3).reshape(B * H, Lq, nt * 64)[:, :, :Lk]
        else:
            n3 = B * H * ((Lq + 31) // 32) * nt * 32
            got = _decode_v3(out[s_, :n3].cpu(), B * H, Lq, Lk)
            # the per-lane dwords (layout v5) that fwd7 / fwd8 / dq7 read: the same bits
            lw = out[s_, n3:2 * n3].cpu()
            dw = torch.stack([lw & 0xFFFFFFFF, (lw >> 32) & 0xFFFFFFFF], -1).reshape(-1)
            ref0 = O.attn_dropout_keep(seed, 7 + 6 * s_, B, H, Lq, Lk, p).reshape(B * H, Lq, Lk)
            got5 = _decode_v5(dw, B * H, Lq, Lk)
            assert torch.equal(got5, ref0), f"site {s_} per-lane dwords: {(got5 != ref0).sum().item()} bits differ"
        ref = O.attn_dropout_keep(seed, 7 + 6 * s_, B, H, Lq, Lk, p).reshape(B * H, Lq, Lk)
        assert torch.equal(got, ref), f"site {s_}: {(got != ref).sum().item()} bits differ"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_attention_relbias(dtype):
    o = ops()
    B, H, S = 2, 2, 75
    D = H * 64
    q = torch.randn(B, S, D, generator=g(30))
    k = torch.randn(B, S, D, generator=g(31))
    v = torch.randn(B, S, D, generator=g(32))
    gate = torch.rand(B, H, S, generator=g(33)) + 1.0
    table = torch.randn(H, 2 * S - 1, generator=g(34))
    to = lambda x: x.to(dev, dtype).reshape(-1, D).contiguous()  # noqa: E731
    od = torch.empty(B * S, D, device=dev, dtype=dtype)
    o.attn_fwd(to(q), to(k), to(v), od, None, B, H, S, S, gate=gate.reshape(B * H, S).to(dev).contiguous(),
               table=table.to(dev))
    hv = lambda x: x.to(dtype).double().view(B, -1, H, 64).transpose(1, 2)  # noqa: E731
    ref = _attn_ref(hv(q), hv(k), hv(v), None, 0.0, 0, 0, gate=gate.double(), table=table.double())
    close(od.float(), ref.transpose(1, 2).reshape(B * S, D), rtol=TOL[dtype], what="relbias attn")


@pytest.mark.parametrize("S", [75, 499])
def test_attention_relgate_matches_gate_kernel_path(S):
    """WavLM attention with the gate computed in the kernel from 8 bf16 pre-activations per (token, head)
    appended to the projection output (fddm_attn_fwd_relgate) vs the two-pass path (fddm_wavlm_gate +
    fddm_attn_fwd) and vs float64 torch on the same bf16 inputs."""
    o = ops()
    B, H, E = 2, 12, 768
    gen = torch.Generator(device=dev).manual_seed(40)
    x = torch.randn(B * S, E, device=dev, generator=gen).bfloat16()
    qkv = torch.randn(B * S, 3 * E, device=dev, generator=gen).bfloat16()
    W = torch.randn(8, 64, device=dev, generator=gen) * 0.2
    bias = torch.randn(8, device=dev, generator=gen) * 0.1
    cst = torch.rand(H, device=dev, generator=gen) + 0.5
    table = torch.randn(H, 2 * S - 1, device=dev, generator=gen)
    # pre-activations as the fused projection produces them (bf16)
    graw = torch.einsum("nhd,od->nho", x.float().view(B * S, H, 64), W) + bias
    buf = torch.zeros(B * S, 3 * E + 8 * H + 8, device=dev, dtype=torch.bfloat16)   # padded row stride
    buf[:, :3 * E] = qkv
    buf[:, 3 * E:3 * E + 8 * H] = graw.reshape(B * S, 8 * H).bfloat16()
    out = torch.empty(B * S, E, device=dev, dtype=torch.bfloat16)
    o.attn_fwd_relgate(buf, buf[:, E:], buf[:, 2 * E:], out, buf[:, 3 * E:], cst, table, B, H, S)
    gate = o.wavlm_gate(x, W, bias, cst, B, S, H)
    out2 = torch.empty_like(out)
    o.attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], out2, None, B, H, S, S, gate=gate, table=table)
    close(out.float(), out2.float(), rtol=2e-2, what="relgate vs gate kernel")
    r = buf[:, 3 * E:3 * E + 8 * H].double().view(B, S, H, 8)
    ga, gb = torch.sigmoid(r[..., :4].sum(-1)), torch.sigmoid(r[..., 4:].sum(-1))
    gref = (ga * (gb * cst.double() - 1) + 2).permute(0, 2, 1)                      # [B, H, S]
    hv = lambda t: t.double().view(B, S, H, 64).transpose(1, 2)  # noqa: E731
    q_, k_, v_ = hv(qkv[:, :E]), hv(qkv[:, E:2 * E]), hv(qkv[:, 2 * E:])
    rel = torch.arange(S, device=dev)[None, :] - torch.arange(S, device=dev)[:, None] + S - 1   # key - query + S-1
    sc = q_ @ k_.transpose(-1, -2) / 8.0 + gref[..., None] * table.double()[:, rel][None]
    ref = torch.softmax(sc, -1) @ v_
    close(out.float(), ref.transpose(1, 2).reshape(B * S, E), rtol=2e-2, what="relgate vs float64")


@pytest.mark.parametrize("S", [499, 70])
def test_attention_relgate_x_matches_gate_kernel_path(S):
    """WavLM attention with the gate computed in the kernel from the attention input x and the folded
    gru_rel_pos_linear weights (fddm_attn_fwd_relgate_x, models/wavlm.py _fold_gate) vs the two-pass path
    (fddm_wavlm_gate + fddm_attn_fwd) and vs float64 torch (per-row pre-activations summed as HF does) on the same
    bf16 inputs; x given with a padded row stride."""
    o = ops()
    from models.wavlm import _fold_gate
    B, H, E = 2, 12, 768
    gen = torch.Generator(device=dev).manual_seed(41)
    xb = torch.randn(B * S, E + 64, device=dev, generator=gen).bfloat16()
    x = xb[:, :E]
    qkv = torch.randn(B * S, 3 * E, device=dev, generator=gen).bfloat16()
    lin = torch.nn.Linear(64, 8).to(dev)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(8, 64, device=dev, generator=gen) * 0.2)
        lin.bias.copy_(torch.randn(8, device=dev, generator=gen) * 0.1)
    cst = torch.rand(H, device=dev, generator=gen) + 0.5
    table = torch.randn(H, 2 * S - 1, device=dev, generator=gen)
    out = torch.empty(B * S, E, device=dev, dtype=torch.bfloat16)
    o.attn_fwd_relgate_x(qkv, qkv[:, E:], qkv[:, 2 * E:], out, x, _fold_gate(lin), cst, table, B, H, S)
    gate = o.wavlm_gate(x.contiguous(), lin.weight.detach(), lin.bias.detach(), cst, B, S, H)
    out2 = torch.empty_like(out)
    o.attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], out2, None, B, H, S, S, gate=gate, table=table)
    close(out.float(), out2.float(), rtol=2e-2, what="relgate_x vs gate kernel")
    r = torch.einsum("nhd,od->nho", x.double().view(B * S, H, 64), lin.weight.detach().double()) + \
        lin.bias.detach().double()
    r = r.view(B, S, H, 8)
    ga, gb = torch.sigmoid(r[..., :4].sum(-1)), torch.sigmoid(r[..., 4:].sum(-1))
    gref = (ga * (gb * cst.double() - 1) + 2).permute(0, 2, 1)                      # [B, H, S]
    hv = lambda t: t.double().view(B, S, H, 64).transpose(1, 2)  # noqa: E731
    q_, k_, v_ = hv(qkv[:, :E]), hv(qkv[:, E:2 * E]), hv(qkv[:, 2 * E:])
    rel = torch.arange(S, device=dev)[None, :] - torch.arange(S, device=dev)[:, None] + S - 1   # key - query + S-1
    sc = q_ @ k_.transpose(-1, -2) / 8.0 + gref[..., None] * table.double()[:, rel][None]
    ref = torch.softmax(sc, -1) @ v_
    close(out.float(), ref.transpose(1, 2).reshape(B * S, E), rtol=2e-2, what="relgate_x vs float64")


@pytest.mark.parametrize("S,src,masked", [(499, "gate", False), (499, "graw", False), (499, "gx", False),
                                          (70, "gx", False), (1000, "gate", False), (203, "gate", True)])
def test_wavlm_attention_fwd7_bias_matches_fwd5_and_float64(S, src, masked):
    """Round 6: WavLM's gated relative-position attention on fwd7's bias build (csrc/attn7.hip REL: the bias slice in
    four shifted LDS copies, the gate from a precomputed row / the projection's 8 extra columns / the attention input)
    against the round-2 fwd5 (fddm_attn_set_kernels(5)) and float64 torch on the same bf16 inputs, for each gate
    source, a ragged key count (70, 203), two key passes past 512 (1000) and a key-padding mask."""
    o = ops()
    from models.wavlm import _fold_gate
    B, H, E = 2, 12, 768
    gen = torch.Generator(device=dev).manual_seed(43 + S)
    x = torch.randn(B * S, E, device=dev, generator=gen).bfloat16()
    qkv = (torch.randn(B * S, 3 * E, device=dev, generator=gen) * 1.5).bfloat16()
    lin = torch.nn.Linear(64, 8).to(dev)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(8, 64, device=dev, generator=gen) * 0.2)
        lin.bias.copy_(torch.randn(8, device=dev, generator=gen) * 0.1)
    cst = torch.rand(H, device=dev, generator=gen) + 0.5
    table = torch.randn(H, 2 * S - 1, device=dev, generator=gen) * 2.0
    keep = None
    if masked:
        keep = torch.ones(B, S, device=dev, dtype=torch.uint8)
        keep[0, S - 37:] = 0
        keep[1, :5] = 0
    gate = o.wavlm_gate(x, lin.weight.detach(), lin.bias.detach(), cst, B, S, H)      # [B*H, S]
    graw = torch.einsum("nhd,od->nho", x.float().view(B * S, H, 64), lin.weight.detach()) + lin.bias.detach()
    buf = torch.zeros(B * S, 3 * E + 8 * H + 8, device=dev, dtype=torch.bfloat16)
    buf[:, :3 * E] = qkv
    buf[:, 3 * E:3 * E + 8 * H] = graw.reshape(B * S, 8 * H).bfloat16()

    def run():
        out = torch.empty(B * S, E, device=dev, dtype=torch.bfloat16)
        if src == "gate":
            o.attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], out, None, B, H, S, S, key_keep=keep, gate=gate, table=table)
        elif src == "graw":
            o.attn_fwd_relgate(buf, buf[:, E:], buf[:, 2 * E:], out, buf[:, 3 * E:], cst, table, B, H, S)
        else:
            o.attn_fwd_relgate_x(qkv, qkv[:, E:], qkv[:, 2 * E:], out, x, _fold_gate(lin), cst, table, B, H, S)
        return out

    new = run()
    old_fam = o.attn_force_kernels("relfwd5")
    try:
        old = run()
    finally:
        o.attn_force_kernels(old_fam)
    close(new.float(), old.float(), rtol=2e-2, what=f"fwd7 bias vs fwd5 ({src})")
    if src == "graw":
        r = buf[:, 3 * E:3 * E + 8 * H].double().view(B, S, H, 8)
    else:
        r = (torch.einsum("nhd,od->nho", x.double().view(B * S, H, 64), lin.weight.detach().double()) +
             lin.bias.detach().double()).view(B, S, H, 8)
    ga, gb = torch.sigmoid(r[..., :4].sum(-1)), torch.sigmoid(r[..., 4:].sum(-1))
    gref = (ga * (gb * cst.double() - 1) + 2).permute(0, 2, 1)                      # [B, H, S]
    if src == "gate":
        gref = gate.double().view(B, H, S)
    hv = lambda t: t.double().view(B, S, H, 64).transpose(1, 2)  # noqa: E731
    q_, k_, v_ = hv(qkv[:, :E]), hv(qkv[:, E:2 * E]), hv(qkv[:, 2 * E:])
    rel = torch.arange(S, device=dev)[None, :] - torch.arange(S, device=dev)[:, None] + S - 1   # key - query + S-1
    sc = q_ @ k_.transpose(-1, -2) / 8.0 + gref[..., None] * table.double()[:, rel][None]
    if keep is not None:
        sc = sc.masked_fill(keep[:, None, None, :] == 0, float("-inf"))
    ref = torch.softmax(sc, -1) @ v_
    close(new.float(), ref.transpose(1, 2).reshape(B * S, E), rtol=2e-2, what=f"fwd7 bias vs float64 ({src})")


# ----------------------------------------------------------------------------- LN / RoPE / embed
@pytest.mark.parametrize("fold", [False, True])
@pytest.mark.parametrize("film", [False, True])
@pytest.mark.parametrize("L", [20, 32])
def test_layernorm_fwd_bwd(film, L, fold):
    """L=32: FiLM rows fall in whole 32-row slabs -> the fused single-pass backward; L=20 with FiLM -> two
    passes (row kernel + column-slab parameter kernel). fold: dgamma / dbeta as slab sums added by one ln_fold
    launch (the decoder block's path; the two-pass form zeroes the partials and adds with atomics), on top of
    nonzero destinations (the fold accumulates, as the atomics do)."""
    o = ops()
    B, d = 3, 192
    N = B * L
    x = torch.randn(N, d, generator=g(40))
    y = torch.randn(N, d, generator=g(41))
    gm = 1 + 0.1 * torch.randn(d, generator=g(42))
    bt = 0.1 * torch.randn(d, generator=g(43))
    fs = 0.2 * torch.randn(B, d, generator=g(44))
    fh = 0.2 * torch.randn(B, d, generator=g(45))
    dout = torch.randn(N, d, generator=g(46))
    p = 0.1
    keep = O.dropout_keep(3, 2, N * d, p).view(N, d).double()
    xr, yr, gr, br, fsr, fhr = (t.double().requires_grad_(True) for t in (x, y, gm, bt, fs, fh))
    s = xr + yr * keep / (1 - p)
    out = F.layer_norm(s, (d,), gr, br, 1e-5)
    if film:
        out = (out.view(B, L, d) * (1 + fsr[:, None]) + fhr[:, None]).view(N, d)
    out.backward(dout.double())
    X = lambda t: t.to(dev).contiguous()  # noqa: E731
    of = torch.empty(N, d, device=dev)
    sv = torch.empty(N, d, device=dev)
    mean = torch.empty(N, device=dev)
    rstd = torch.empty(N, device=dev)
    o.ln_fwd(X(x), X(y), X(gm), X(bt), out_f32=of, save_s=sv, mean=mean, rstd=rstd,
             film=(X(fs), X(fh)) if film else None, rows_per_batch=L, drop_p=p, seed=3, rng_stream=2)
    dres = torch.empty(N, d, device=dev)
    dy = torch.empty(N, d, device=dev)
    base = torch.linspace(-1, 1, d, device=dev) if fold else torch.zeros(d, device=dev)
    dg, db = base.clone(), 2 * base
    dfs, dfh = torch.zeros(B, d, device=dev), torch.zeros(B, d, device=dev)
    lnp = o.LnPartials() if fold else None
    o.ln_bwd(X(dout), sv, mean, rstd, X(gm), X(bt), dres=dres, dy_t=dy, dgamma=dg, dbeta=db,
             film_scale=X(fs) if film else None, dfilm=(dfs, dfh) if film else None, rows_per_batch=L, drop_p=p,
             seed=3, rng_stream=2, partials=lnp)
    if fold:
        lnp.fold()
    close(of, out.detach(), rtol=1e-5, what="ln out")
    close(dres, xr.grad, rtol=1e-4, what="ln dx")
    close(dy, yr.grad, rtol=1e-4, what="ln dy")
    close(dg - base, gr.grad, rtol=1e-4, what="dgamma")
    close(db - 2 * base, br.grad, rtol=1e-4, what="dbeta")
    if film:
        close(dfs, fsr.grad, rtol=1e-4, what="dfilm scale")
        close(dfh, fhr.grad, rtol=1e-4, what="dfilm shift")


@pytest.mark.parametrize("d", [512, 768])
def test_ln_fwd_rope_handoff_matches_rope_fwd(d):
    """The decoder LN3's fused RoPE output (the next block's q = k input) equals rope_fwd of the LN's own f32
    output (the unfused path), rounded to bf16: at most one bf16 ulp apart (an FMA contraction may differ), on
    rows of several positions (N = 3 L, L = 37) at the decoder's d = 512 (one chunk per lane) and 768 (two)."""
    o = ops()
    L, N = 37, 111
    x = torch.randn(N, d, generator=g(56)).to(dev)
    y = torch.randn(N, d, generator=g(57)).to(torch.bfloat16).to(dev)
    gm = (1 + 0.1 * torch.randn(d, generator=g(58))).to(dev)
    bt = (0.1 * torch.randn(d, generator=g(59))).to(dev)
    cos, sin = O.rope_cos_sin(L, O.rope_inv_freq(d))
    cos, sin = cos.to(dev).contiguous(), sin.to(dev).contiguous()
    of = torch.empty(N, d, device=dev)
    ot = torch.empty(N, d, device=dev, dtype=torch.bfloat16)
    xr = torch.empty(N, d, device=dev, dtype=torch.bfloat16)
    o.ln_fwd(x, y, gm, bt, out_f32=of, out_t=ot, drop_p=0.1, seed=5, rng_stream=6, rope=(cos, sin, xr, L))
    ref = torch.empty(N, d, device=dev, dtype=torch.bfloat16)
    o.rope_fwd(of, cos, sin, ref, L)
    ulp = (xr.float() - ref.float()).abs() / ref.float().abs().clamp_min(1e-30)
    assert (ulp <= 2.0 ** -7).all(), f"rope hand-off vs rope_fwd: max rel {ulp.max().item():.2e}"
    assert (xr == ref).float().mean().item() > 0.99


@pytest.mark.parametrize("N,d", [(1001, 768), (37, 200), (64, 1024)])
def test_ln_fwd_bf16_post_ln_rows(N, d):
    """The frozen encoder's post-LN (bf16 x + bf16 residual -> bf16, one row per wave, 2 chunks of 8 per lane):
    ragged row counts (N % 4 != 0), d with fewer chunks than lanes (200) and the largest d (1024), against a float64
    layer_norm of the same bf16 inputs within the bf16 output rounding (2^-8 relative + 1e-3)."""
    o = ops()
    bf = torch.bfloat16
    x = torch.randn(N, d, generator=g(47)).to(bf)
    y = (0.5 * torch.randn(N, d, generator=g(48)) + 0.3).to(bf)
    gm = 1 + 0.1 * torch.randn(d, generator=g(42))
    bt = 0.1 * torch.randn(d, generator=g(43))
    ref = F.layer_norm(x.double() + y.double(), (d,), gm.double(), bt.double(), 1e-5)
    out = torch.empty(N, d, device=dev, dtype=bf)
    mean = torch.empty(N, device=dev)
    rstd = torch.empty(N, device=dev)
    o.ln_fwd(x.to(dev), y.to(dev), gm.to(dev), bt.to(dev), out_t=out, mean=mean, rstd=rstd, eps=1e-5)
    err = (out.double().cpu() - ref).abs()
    assert (err <= 2.0 ** -8 * ref.abs() + 1e-3).all(), float(err.max())
    s = x.double() + y.double()
    close(mean, s.mean(1), rtol=1e-5, what="mean")
    close(rstd, 1 / torch.sqrt(s.var(1, unbiased=False) + 1e-5), rtol=1e-4, what="rstd")


@pytest.mark.parametrize("B,L,d,n", [(2, 100, 512, 1024), (1, 256, 256, 512), (3, 50, 128, 256)])
def test_linear_dx_rope_matches_gemm_then_rope_bwd(B, L, d, n):
    """fddm_linear_dx_rope (gemm128 EPI_ROPE_ACC: dx += rope_bwd(dy @ w), RoPE partner columns j, j + d/2 loaded into
    one tile) against float64: dy @ w, then the oracle's RoPE backward by autograd, added to a random dx. Ragged row
    counts (200, 150) exercise the overlapping last tile."""
    o = ops()
    M = B * L
    inv = O.rope_inv_freq(d)
    cos, sin = O.rope_cos_sin(L, inv)
    dy = torch.randn(M, n, generator=g(60)).to(torch.bfloat16)
    w = (torch.randn(n, d, generator=g(61)) / math.sqrt(n)).to(torch.bfloat16)
    dx0 = torch.randn(M, d, generator=g(62))
    dx = dx0.to(dev)
    assert o.linear_dx_rope(dy.to(dev), w.to(dev), dx, cos.to(dev).contiguous(), sin.to(dev).contiguous(), L)
    xr = torch.zeros(B, L, d, dtype=torch.float64, requires_grad=True)
    ref = O.rope_apply(xr, cos.double(), sin.double())
    ref.backward((dy.double() @ w.double()).view(B, L, d))
    close(dx, dx0.double() + xr.grad.view(M, d), rtol=1e-5, what="dx += rope_bwd(dy w)")


@pytest.mark.parametrize("d", [128, 6])
def test_rope_and_embedding(d):
    """d = 128: the vectorised kernels (8 columns per thread); d = 6: the scalar forms."""
    o = ops()
    B, L, V = 2, 9, 50
    inv = O.rope_inv_freq(d)
    cos, sin = O.rope_cos_sin(L, inv)
    x = torch.randn(B * L, d, generator=g(50))
    out = torch.empty(B * L, d, device=dev)
    o.rope_fwd(x.to(dev), cos.to(dev), sin.to(dev), out, L)
    xr = x.view(B, L, d).double().requires_grad_(True)
    ref = O.rope_apply(xr, cos.double(), sin.double())
    close(out.view(B, L, d), ref.detach(), rtol=1e-6, what="rope")
    dy = torch.randn(B, L, d, generator=g(51)).double()
    ref.backward(dy)
    dx = torch.zeros(B * L, d, device=dev)
    o.rope_bwd(dy.float().view(-1, d).to(dev), cos.to(dev), sin.to(dev), dx, L)
    close(dx.view(B, L, d), xr.grad, rtol=1e-5, what="rope bwd")
    tok = torch.randint(0, V, (B, L), generator=g(52))
    tok[1, -3:] = 0
    E = torch.randn(V, d, generator=g(53))
    tb = torch.randn(B, d, generator=g(54))
    xo = torch.empty(B * L, d, device=dev)
    o.embed_fwd(tok.to(dev), E.to(dev), tb.to(dev), xo, None, L)
    close(xo.view(B, L, d), E[tok] + tb[:, None], rtol=1e-6, what="embed")
    dxe = torch.randn(B * L, d, generator=g(55))
    dE = torch.zeros(V, d, device=dev)
    dtb = torch.zeros(B, d, device=dev)
    o.embed_bwd(tok.to(dev).reshape(-1), dxe.to(dev), dE, dtb, L, 0)
    refE = torch.zeros(V, d).index_add_(0, tok.reshape(-1), dxe)
    refE[0] = 0
    close(dE, refE, rtol=1e-5, what="dE")
    close(dtb, dxe.view(B, L, d).sum(1), rtol=1e-5, what="dtbias")


# ---------------------------------------------------------------------------- diffusion kernels
def test_sampler_bit_exact_and_kl():
    o = ops()
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    K, Tn, B, L = 8000, 200, 16, 256
    sch = DiscreteDiffusionScheduler(K=K, T=Tn, device=dev)
    x0 = torch.randint(1, K, (B, L), generator=g(60))
    t = torch.randint(1, Tn + 1, (B,), generator=g(61))
    t[0], t[1] = 1, 2
    xt = sch.sample_xt(x0.to(dev), t.to(dev), seed=1234)
    _, ab = O.sched_tables(Tn)
    ref = O.sample_xt(x0, t, K, ab, seed=1234, stream=1)
    assert torch.equal(xt.cpu(), ref), "sampled indices must be bit-exact"
    # fused KL forward/backward vs closed form oracle (and fixture-pinned formula)
    from helpers import load, T
    gk = load("kl")
    logits, xtk, x0k, tk, xm, betas = (T(gk[n]) for n in ("logits", "xt", "x0", "t", "x_mask", "betas"))
    Bk, Lk, Vk = logits.shape
    valid = xm.float()
    w = (valid / (valid.sum(1, keepdim=True) + 1e-8) / Bk).reshape(-1)
    kl_tok = o.kl_fwd(logits.view(-1, Vk).to(dev), xtk.reshape(-1).to(dev), x0k.reshape(-1).to(dev), tk.to(dev),
                      betas.to(dev), Lk)
    loss = (kl_tok.cpu() * w).sum()
    close(loss, gk["kl"], rtol=1e-5, what="kl loss")
    gs = torch.full((1,), 2.0, device=dev)
    dz = o.kl_bwd(logits.view(-1, Vk).to(dev), xtk.reshape(-1).to(dev), x0k.reshape(-1).to(dev), tk.to(dev),
                  betas.to(dev), w.to(dev), gs, Lk)
    close(dz.view(Bk, Lk, Vk), 2 * T(gk["dlogits"]), rtol=1e-4, atol=1e-10, what="kl grad")


def test_kl_full_vocab_matches_oracle():
    """C2 vocabulary (V=8000): the kernel's generic-index form with the x_t / x0 corrections vs the closed form
    over every index (oracle, fp32), incl. t=1 (beta_p = 0), t=T, x_t == x0 rows and a masked row."""
    o = ops()
    K, Tn, B, L = 8000, 200, 4, 256
    betas, _ = O.sched_tables(Tn)
    logits = 3.0 * torch.randn(B, L, K, generator=g(70))
    x0 = torch.randint(1, K, (B, L), generator=g(71))
    xt = torch.randint(1, K, (B, L), generator=g(72))
    xt[:, ::3] = x0[:, ::3]
    t = torch.tensor([1, 2, 117, 200])
    xm = torch.ones(B, L, dtype=torch.bool)
    xm[2, 200:] = False
    ref_loss, ref_dz = O.kl_term(logits, xt, x0, t, xm, betas)
    valid = xm.float()
    w = (valid / (valid.sum(1, keepdim=True) + 1e-8) / B).reshape(-1)
    kl_tok = o.kl_fwd(logits.view(-1, K).to(dev), xt.reshape(-1).to(dev), x0.reshape(-1).to(dev), t.to(dev),
                      betas.to(dev), L)
    close((kl_tok.cpu() * w).sum(), ref_loss, rtol=1e-4, what="kl loss V=8000")
    dz = o.kl_bwd(logits.view(-1, K).to(dev), xt.reshape(-1).to(dev), x0.reshape(-1).to(dev), t.to(dev),
                  betas.to(dev), w.to(dev), None, L)
    err = (dz.view(B, L, K).cpu() - ref_dz).abs().max() / ref_dz.abs().max()
    assert err < 1e-4, f"kl grad V=8000 rel err {err:.2e}"


@pytest.mark.parametrize("scale", [3.0, 30.0])
def test_kl_fused_matches_oracle_and_scale_if(scale):
    """The train step's one-pass KL (kl_tok + w-weighted gradient, w from the mask in the kernel) vs the closed-form
    oracle: loss within 1e-4, f32 gradient within 1e-4 of the max, bf16 gradient within bf16 rounding (2^-8
    relative per element + 1e-4 of the max); unmasked (plain mean) too; scale_if applies g != 1, skips g == 1.
    scale 30: peaked rows, so at t = 1 (beta_p = 0) nearly every P + eps sits at eps = 1e-8 — the floor of the
    kernel's one-log-per-four product (4 factors >= 1e-8: >= 1e-32, still a normal f32)."""
    o = ops()
    K, Tn, B, L = 8000, 200, 4, 256
    betas, _ = O.sched_tables(Tn)
    logits = scale * torch.randn(B, L, K, generator=g(73))
    x0 = torch.randint(1, K, (B, L), generator=g(74))
    xt = torch.randint(1, K, (B, L), generator=g(75))
    xt[:, ::3] = x0[:, ::3]
    t = torch.tensor([1, 2, 117, 200])
    for masked in (True, False):
        xm = torch.ones(B, L, dtype=torch.bool)
        if masked:
            xm[2, 200:] = False
            xm[0, 17] = False
        ref_loss, ref_dz = O.kl_term(logits, xt, x0, t, xm if masked else None, betas)
        args = (logits.view(-1, K).to(dev), xt.reshape(-1).to(dev), x0.reshape(-1).to(dev), t.to(dev), betas.to(dev),
                xm.reshape(-1).to(dev).view(torch.uint8) if masked else None, L)
        for dt in (torch.float32, torch.bfloat16):
            kl_tok, dz = o.kl_fused(*args, out_dtype=dt)
            loss, _ = o.kl_reduce(kl_tok, args[5], B, L, want_w=False)
            close(loss, ref_loss, rtol=1e-4, what=f"fused kl loss masked={masked}")
            d = dz.float().view(B, L, K).cpu()
            tol = 1e-4 * ref_dz.abs().max() + (2.0 ** -8 * ref_dz.abs() if dt == torch.bfloat16 else 0.0)
            bad = ((d - ref_dz).abs() > tol).sum().item()
            assert bad == 0, f"fused kl grad {dt} masked={masked}: {bad} elements off"
            before = dz.clone()
            o.scale_if(dz, torch.ones(1, device=dev))
            assert torch.equal(dz, before)
            o.scale_if(dz, torch.full((1,), -3.0, device=dev))
            close(dz.float(), -3.0 * before.float(), rtol=1e-2 if dt == torch.bfloat16 else 1e-6, what="scale_if")


def test_lfd_kernels_match_reference():
    from helpers import load, T
    from fddm_hip import runtime as rt
    from losses.fddm_losses import lfd_loss
    gl = load("lfd")
    with rt.use_precision("fp32"):
        za = T(gl["za"]).to(dev).requires_grad_(True)
        zb = T(gl["zb"]).to(dev).requires_grad_(True)
        loss = lfd_loss(za, zb, 5e-3)
        loss.backward()
    close(loss, gl["loss"], rtol=1e-5, what="lfd")
    close(za.grad, gl["dza"], rtol=1e-4, what="dza")
    close(zb.grad, gl["dzb"], rtol=1e-4, what="dzb")


def test_fused_adamw_matches_oracle():
    from fddm_hip.optim import FusedAdamW
    from fddm_hip import runtime as rt
    torch.manual_seed(0)
    shapes = [(300, 70), (70,), (1000,)]
    ps = [torch.randn(*s) for s in shapes]
    with rt.use_precision("fp32"):
        dps = [torch.nn.Parameter(p.clone().to(dev)) for p in ps]
        opt = FusedAdamW(dps, lr=2e-4, weight_decay=0.01)
        ref = {str(i): p.clone() for i, p in enumerate(ps)}
        ro = O.OracleAdamW()
        for step in range(3):
            grads = [10 * torch.randn(*s) for s in shapes]
            skip = step == 1
            for i, (p, gr) in enumerate(zip(dps, grads)):
                p.grad = None if (skip and i == 2) else gr.to(dev)
            opt.clip_and_step(max_norm=5.0)
            gd = {str(i): (None if (skip and i == 2) else grads[i].clone()) for i in range(3)}
            O.clip_grads(gd, 5.0)
            ro.step(ref, gd)
    for i, p in enumerate(dps):
        close(p, ref[str(i)], rtol=1e-5, atol=1e-7, what=f"adamw p{i}")


def test_softmax_rows_and_bwd():
    o = ops()
    x = 3 * torch.randn(37, 1000, generator=g(70))
    y = o.softmax_rows(x.to(dev), torch.float32)
    close(y, torch.softmax(x.double(), -1), rtol=1e-5, what="softmax")
    dy = torch.randn(37, 1000, generator=g(71))
    dz = o.softmax_bwd_rows(y, dy.to(dev))
    yr = torch.softmax(x.double(), -1)
    ref = yr * (dy.double() - (yr * dy.double()).sum(-1, keepdim=True))
    close(dz, ref, rtol=1e-5, what="softmax bwd")


@pytest.mark.parametrize("V", [8000, 1000, 24])
def test_softmax_bwd_add_bf16_and_axpy_if(V):
    """The bf16 hand-over kernels: y*(dy - rowsum(y*dy)) + add from bf16 operands (f32 arithmetic, one bf16
    rounding of the result: within 2^-8 relative + 1e-3 of the row scale), in place over `add` too; axpy_if adds
    (g-1)*y and leaves x untouched bit for bit when g == 1."""
    o = ops()
    bf = torch.bfloat16
    N = 19
    x = 3 * torch.randn(N, V, generator=g(76))
    y = torch.softmax(x, -1).to(bf)
    dy = torch.randn(N, V, generator=g(77)).to(bf)
    add = (1e-3 * torch.randn(N, V, generator=g(78))).to(bf)
    yd, dyd = y.double(), dy.double()
    ref = yd * (dyd - (yd * dyd).sum(-1, keepdim=True)) + add.double()
    out = o.softmax_bwd_add_bf16(y.to(dev), dy.to(dev), add.to(dev)).cpu().double()
    tol = 2.0 ** -8 * ref.abs() + 1e-3 * ref.abs().amax(-1, keepdim=True)
    assert ((out - ref).abs() <= tol).all()
    a = add.to(dev)
    o.softmax_bwd_add_bf16(y.to(dev), dy.to(dev), a, out=a)
    assert torch.equal(a.cpu().double(), out)
    xb = torch.randn(N * V, generator=g(79)).to(bf).to(dev)
    yb = torch.randn(N * V, generator=g(80)).to(bf).to(dev)
    before = xb.clone()
    o.axpy_if_bf16(xb, yb, torch.ones(1, device=dev))
    assert torch.equal(xb, before)
    o.axpy_if_bf16(xb, yb, torch.full((1,), 3.0, device=dev))
    close(xb.float(), before.float() + 2.0 * yb.float(), rtol=1e-2, atol=1e-2, what="axpy_if")


def test_fused_adamw_nonfinite_guard_skips_whole_step():
    """A non-finite gradient norm skips the whole step on the device — parameters, moments and the step
    counters stay as they were (GradScaler.step's skip on the reference's GPU path, train.py:401-413) — and the
    next finite step continues exactly as if the skipped one never happened."""
    from fddm_hip.optim import FusedAdamW
    from fddm_hip import runtime as rt
    torch.manual_seed(1)
    shapes = [(64, 33), (33,)]
    ps = [torch.randn(*s) for s in shapes]
    grads = [[10 * torch.randn(*s) for s in shapes] for _ in range(3)]
    grads[1][0][3, 5] = float("nan")
    with rt.use_precision("fp32"):
        dps = [torch.nn.Parameter(p.clone().to(dev)) for p in ps]
        opt = FusedAdamW(dps, lr=2e-4, weight_decay=0.01)
        ref = {str(i): p.clone() for i, p in enumerate(ps)}
        ro = O.OracleAdamW()
        for step in range(3):
            for p, gr in zip(dps, grads[step]):
                p.grad = gr.to(dev)
            opt.clip_and_step(max_norm=5.0)
            if step == 1:
                torch.cuda.synchronize()
                assert int(opt.skipped_steps()[0]) == 1
                assert all(float(opt.state[p]["step"]) == 1.0 for p in dps)
                continue
            gd = {str(i): grads[step][i].clone() for i in range(2)}
            O.clip_grads(gd, 5.0)
            ro.step(ref, gd)
    for i, p in enumerate(dps):
        close(p, ref[str(i)], rtol=1e-5, atol=1e-7, what=f"guarded adamw p{i}")
    assert all(float(opt.state[p]["step"]) == 2.0 for p in dps)


@pytest.mark.parametrize("finite", [True, False])
def test_fused_adamw_zero_grads_in_step(finite):
    """clip_and_step(zero_grads=True) (the train loop's form: the grad arena's zero fill folded into AdamW's read of it)
    updates parameters and moments exactly as the plain step and leaves every gradient zero — also when the non-finite
    guard skips the update — so the next zero_grad skips the arena fill."""
    from fddm_hip.optim import FusedAdamW
    from fddm_hip import runtime as rt
    torch.manual_seed(4)
    shapes = [(257, 33), (33,), (1000,)]
    init = [torch.randn(*s_) for s_ in shapes]
    grads = [10 * torch.randn(*s_) for s_ in shapes]
    if not finite:
        grads[0][5, 7] = float("nan")
    out = []
    with rt.use_precision("fp32"):
        for zg in (False, True):
            ps = [torch.nn.Parameter(x.clone().to(dev)) for x in init]
            opt = FusedAdamW(ps, lr=2e-4, weight_decay=0.01)
            arena = opt.use_grad_arena(ps)
            opt.zero_grad()
            for p_, g_ in zip(ps, grads):
                p_.grad.copy_(g_.to(dev))
            opt.clip_and_step(max_norm=5.0, zero_grads=zg)
            torch.cuda.synchronize()
            out.append([p_.detach().cpu().clone() for p_ in ps])
            if zg:
                assert arena.clean and float(arena.flat.abs().max()) == 0.0
                opt.zero_grad()
                assert not arena.clean and all(p_.grad.data_ptr() == v.data_ptr() for p_, v in zip(ps, arena.views))
            else:
                assert float(arena.flat.abs().max()) > 0 or not finite
    for a_, b_ in zip(*out):
        assert torch.equal(a_, b_)


def test_fused_adamw_skip_counts_once_over_groups():
    """With several parameter groups a skipped (non-finite) step is counted once, not once per group's launch
    (ADVICE r2), and no group is updated."""
    from fddm_hip.optim import FusedAdamW
    from fddm_hip import runtime as rt
    with rt.use_precision("fp32"):
        ps = [torch.nn.Parameter(torch.randn(40, 7, device=dev)) for _ in range(3)]
        opt = FusedAdamW([{"params": [ps[0]]}, {"params": [ps[1]], "lr": 1e-3}, {"params": [ps[2]]}], lr=2e-4)
        before = [p.detach().clone() for p in ps]
        for p in ps:
            p.grad = torch.randn(40, 7, device=dev)
        ps[1].grad[0, 0] = float("inf")
        opt.clip_and_step(max_norm=5.0)
        torch.cuda.synchronize()
        assert int(opt.skipped_steps()[0]) == 1
        assert all(torch.equal(p.detach(), b) for p, b in zip(ps, before))


def test_fused_adamw_follows_replaced_bf16_copies():
    """The optimizer writes each weight's bf16 copy for the next forward; when the runtime cache replaces that
    copy (clear_cache after a checkpoint load, an in-place change of the parameter), the optimizer's device
    table must follow the live copy instead of writing the old buffer (stale pointer)."""
    from fddm_hip.optim import FusedAdamW
    from fddm_hip import runtime as rt
    torch.manual_seed(2)
    with rt.use_precision("bf16"):
        w = torch.nn.Parameter(torch.randn(128, 96, device=dev))
        opt = FusedAdamW([w], lr=1e-2)
        rt.wt(w)
        for step in range(3):
            w.grad = torch.randn(128, 96, device=dev)
            opt.clip_and_step(max_norm=None)
            if step == 0:
                rt.clear_cache()
                rt.wt(w)                    # the forward's new bf16 copy
            if step == 1:
                with torch.no_grad():
                    w.mul_(0.5)             # version bump: the next forward re-casts
                rt.wt(w)
            torch.cuda.synchronize()
            assert torch.equal(rt.wt(w), w.detach().to(torch.bfloat16)), f"step {step}"


# ------------------------------------------------------------------------------ small per-batch ops
def test_small_linear_and_dw_match_torch():
    """csrc/small.hip: the time-MLP / FiLM Linears (one launch for several weight sets, SiLU fused, transposed
    weights for input gradients, SiLU' fused) and their weight / bias gradients vs float64 torch."""
    o = ops()
    gen = torch.Generator().manual_seed(40)
    R, K, N = 32, 96, 200
    x = torch.randn(R, K, generator=gen)
    Ws = [torch.randn(N, K, generator=gen) / 10 for _ in range(3)]
    bs = [torch.randn(N, generator=gen) for _ in range(3)]
    outs = [torch.empty(R, N, device=dev) for _ in range(3)]
    o.small_linear(x.to(dev), [w.to(dev) for w in Ws], [b.to(dev) for b in bs], outs)
    for w, b, out in zip(Ws, bs, outs):
        close(out, x.double() @ w.double().T + b.double(), rtol=1e-5, what="small_linear")
    pre, act = torch.empty(R, N, device=dev), torch.empty(R, N, device=dev)
    o.small_linear(x.to(dev), [Ws[0].to(dev)], [bs[0].to(dev)], [pre], [act], act=1)
    ref = x.double() @ Ws[0].double().T + bs[0].double()
    close(pre, ref, rtol=1e-5, what="pre")
    close(act, torch.nn.functional.silu(ref), rtol=1e-5, what="silu")
    dy = torch.randn(R, N, generator=gen)
    dx = torch.empty(R, K, device=dev)
    o.small_linear(dy.to(dev), [Ws[1].to(dev)], None, [dx], transpose_w=True)
    close(dx, dy.double() @ Ws[1].double(), rtol=1e-5, what="dx")
    aux = torch.randn(R, K, generator=gen)
    dxs = torch.empty(R, K, device=dev)
    o.small_linear(dy.to(dev), [Ws[1].to(dev)], None, [dxs], act=2, aux=aux.to(dev), transpose_w=True)
    sg = torch.sigmoid(aux.double())
    close(dxs, (dy.double() @ Ws[1].double()) * sg * (1 + aux.double() * (1 - sg)), rtol=1e-5, what="dsilu")
    # >= 128 tiles of 32 columns: the register-tile kernel (linrt), with ragged rows (45), K (96) and columns (400)
    R3, K3, N3, nj = 45, 96, 400, 12
    x3 = torch.randn(R3, K3, generator=gen)
    W3 = [torch.randn(N3, K3, generator=gen) / 10 for _ in range(nj)]
    b3 = [torch.randn(N3, generator=gen) for _ in range(nj)]
    o3, o3s = [torch.empty(R3, N3, device=dev) for _ in range(nj)], [torch.empty(R3, N3, device=dev) for _ in range(nj)]
    o.small_linear(x3.to(dev), [w.to(dev) for w in W3], [b.to(dev) for b in b3], o3, o3s, act=1)
    for w, b, out, outs in zip(W3, b3, o3, o3s):
        ref = x3.double() @ w.double().T + b.double()
        close(out, ref, rtol=1e-5, what="small_linear (tiles)")
        close(outs, torch.nn.functional.silu(ref), rtol=1e-5, what="silu (tiles)")
    WT = [torch.randn(K3, N3, generator=gen) / 10 for _ in range(nj)]
    aux3 = torch.randn(R3, N3, generator=gen)
    oT = [torch.empty(R3, N3, device=dev) for _ in range(nj)]
    o.small_linear(x3.to(dev), [w.to(dev) for w in WT], None, oT, act=2, aux=aux3.to(dev), transpose_w=True)
    sg3 = torch.sigmoid(aux3.double())
    for w, out in zip(WT, oT):
        close(out, (x3.double() @ w.double()) * sg3 * (1 + aux3.double() * (1 - sg3)), rtol=1e-5, what="dsilu (tiles)")
    dW = [torch.full((N, K), 0.5, device=dev) for _ in range(2)]
    db = [torch.full((N,), 0.25, device=dev) for _ in range(2)]
    xs = [torch.randn(R, K, generator=gen) for _ in range(2)]
    dys = [torch.randn(R, N, generator=gen) for _ in range(2)]
    o.small_dw([(dys[i].to(dev), xs[i].to(dev), dW[i], db[i]) for i in range(2)])
    for i in range(2):
        close(dW[i], 0.5 + dys[i].double().T @ xs[i].double(), rtol=1e-5, what="small_dw")
        close(db[i], 0.25 + dys[i].double().sum(0), rtol=1e-5, what="small_db")
    # 45 rows (two row chunks of the kernel), K a multiple of 4 and not
    for K2 in (96, 98):
        R2 = 45
        x2, dy2 = torch.randn(R2, K2, generator=gen), torch.randn(R2, N, generator=gen)
        dW2, db2 = torch.zeros(N, K2, device=dev), torch.zeros(N, device=dev)
        o.small_dw([(dy2.to(dev), x2.to(dev), dW2, db2)])
        close(dW2, dy2.double().T @ x2.double(), rtol=1e-5, what=f"small_dw K={K2}")
        close(db2, dy2.double().sum(0), rtol=1e-5, what=f"small_db K={K2}")


def test_rows_mean_time_embed_kl_reduce():
    o = ops()
    gen = torch.Generator().manual_seed(41)
    x = torch.randn(3, 37, 130, generator=gen)
    for dt in (torch.float32, torch.bfloat16):
        xd = x.to(dev, dt)
        close(o.rows_mean(xd), xd.double().mean(1), rtol=1e-6, what=f"rows_mean {dt}")
    t = torch.tensor([1, 7, 200, 55])
    # sin/cos of t * f with t up to T = 200: a 1-ulp difference of f between the device expf and the CPU's exp
    # moves the argument by up to 200 * 6e-8, hence the 3e-5 absolute tolerance
    close(o.time_embed(t.to(dev), 512, 10000), O.time_embedding(t, 512), rtol=0, atol=3e-5, what="time_embed")
    close(o.time_embed(t.to(dev), 129, 10000), O.time_embedding(t, 129), rtol=0, atol=3e-5, what="time_embed odd")
    B, L = 5, 70
    kl = torch.rand(B * L, generator=gen)
    m = torch.rand(B, L, generator=gen) > 0.3
    m[3] = False                                  # an all-pad row: per = 0 / (0 + eps)
    loss, w = o.kl_reduce(kl.to(dev), m.reshape(-1).to(dev).view(torch.uint8), B, L)
    v = m.double()
    per = (kl.view(B, L).double() * v).sum(1) / (v.sum(1) + 1e-8)
    close(loss, per.mean(), rtol=1e-6, what="kl_reduce loss")
    close(w.view(B, L), v / (v.sum(1, keepdim=True) + 1e-8) / B, rtol=1e-6, what="kl_reduce w")
    loss2, w2 = o.kl_reduce(kl.to(dev), None, B, L)
    close(loss2, kl.double().mean(), rtol=1e-6, what="kl_reduce unmasked")
    close(w2, torch.full((B * L,), 1.0 / (B * L)), rtol=1e-6, what="kl_reduce unmasked w")


def test_conv0_gn_gelu_matches_reference():
    """WavLM conv layer 0 + per-channel GroupNorm over time + GELU (HF modeling_wavlm.py:723-744) in bf16 (Gram-
    matrix statistics; the bf16 output's conv + affine on the matrix cores as a hi/lo bf16 split, the f32 output's
    on the VALU) vs a float64 torch reference within bf16 rounding (2^-8 relative + 2e-3 absolute) resp. 1e-4;
    16007 samples = 3200 frames, 12345 = 2468 frames (ragged 512-frame blocks and 16-frame tiles), 45007 = 9000 frames
    (three 4096-frame statistics blocks, the last one ragged: the per-block partial statistics summed in a fixed
    order by the affine kernel; the 10 s training input has eight)."""
    o = ops()
    C, K, S = 512, 10, 5
    w = torch.randn(C, K, generator=g(82)) * 0.3
    gamma = 1 + 0.1 * torch.randn(C, generator=g(83))
    beta = 0.1 * torch.randn(C, generator=g(84))
    for B, nsamp in ((3, 16000 + 7), (2, 12345), (2, 45007)):
        wave = torch.randn(B, nsamp, generator=g(81)) * 0.1
        y = F.conv1d(wave.double()[:, None], w.double()[:, None], stride=S)            # [B, C, T]
        y = F.group_norm(y, C, gamma.double(), beta.double(), eps=1e-5)
        ref = F.gelu(y).transpose(1, 2)
        out = o.conv0_gn_gelu(wave.to(dev), w.to(dev), gamma.to(dev), beta.to(dev), torch.bfloat16, C, K, S)
        out = out.float().cpu()
        assert ref.shape == out.shape
        err = (out.double() - ref).abs()
        assert (err <= 2.0 ** -8 * ref.abs() + 2e-3).all(), float(err.max())
        # the conv itself at f32-level accuracy: outputs whose exact value is far from a bf16 rounding boundary
        # agree with the rounded exact value to within one bf16 ulp
        assert (err <= 2.0 ** -7 * ref.abs() + 1e-4).float().mean() > 0.999
        out32 = o.conv0_gn_gelu(wave.to(dev), w.to(dev), gamma.to(dev), beta.to(dev), torch.float32, C, K, S).cpu()
        assert ((out32.double() - ref).abs() <= 1e-4 * ref.abs() + 1e-5).all()
