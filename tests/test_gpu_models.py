"""Module-level GPU parity: the drop-in modules (fddm-asr_amd/) against the reference's golden
fixtures and the CPU oracle, in the exact-fp32 parity mode (1e-4 relative), plus bf16-mode sanity.
"""
import numpy as np
import pytest
import torch

from helpers import SMALL_WAVLM, T, _dec_sd, _step_params, close, load, wavlm_sd
from oracle import fddm_oracle as O

pytestmark = pytest.mark.gpu
dev = torch.device("cuda:0")


def _rt():
    from fddm_hip import runtime as rt
    return rt


def make_decoder(V, d, H, NL, FF, dropout=0.0):
    from models.denoise_decoder import DenoisingTransformerDecoder
    dec = DenoisingTransformerDecoder(vocab_size=V, d_model=d, nhead=H, num_layers=NL, dim_ff=FF, dropout=dropout,
                                      max_len=1024, pad_id=0)
    sd = dec.state_dict()
    for n, v in _dec_sd(V, d, H, NL, FF).items():
        sd[n] = v
    dec.load_state_dict(sd)
    return dec.to(dev)


def test_decoder_fp32_matches_reference_fixture():
    g = load("decoder")
    rt = _rt()
    with rt.use_precision("fp32"):
        dec = make_decoder(1000, 128, 2, 2, 256)
        dec.train()
        cond = T(g["cond"]).to(dev)
        logits = dec(T(g["xt"]).to(dev), T(g["t"]).to(dev), cond, x_mask=T(g["x_mask"]).to(dev))
        close(logits, g["logits"], rtol=1e-4, what="decoder logits")
        (logits * T(g["R"]).to(dev)).sum().backward()
        for n, p in dec.named_parameters():
            if "g." + n in g:
                close(p.grad, g["g." + n], rtol=1e-4, atol=1e-6, what="grad " + n)
            close((p.grad.double() ** 2).sum(), g["g_sq." + n], rtol=2e-4, what="grad sq " + n)
        with torch.no_grad():
            l2 = dec(T(g["xt"]).to(dev), T(g["t"]).to(dev), cond)
        close(l2, g["logits_defmask"], rtol=1e-4, what="decoder default mask")


@pytest.mark.parametrize("prec,tol,H,d", [("fp32", 1e-4, 2, 128), ("bf16", 3e-2, 2, 128), ("fp32", 1e-4, 4, 128),
                                          ("bf16", 3e-2, 4, 128), ("fp32", 1e-4, 8, 128), ("bf16", 3e-2, 4, 200)])
def test_decoder_dropout_matches_oracle(prec, tol, H, d, monkeypatch):
    """Dropout 0.1 everywhere: masks follow the shared RNG contract, so GPU == oracle. H = 4 / 8 are head_dim
    32 / 16 (C1's d_model 128 with 4 heads): the kernels run them on zero-padded 64-wide head slots. d = 200
    (d % 16 == 8, head_dim 50): the bf16 LN3 -> next block RoPE hand-off is not taken (the fused kernel needs d % 16
    == 0), the blocks run their own rope_fwd."""
    rt = _rt()
    V, NL, FF, B, L, S = 304, 2, 256, 2, 24, 30
    gen = torch.Generator().manual_seed(3)
    xt = torch.randint(1, V, (B, L), generator=gen)
    xt[1, 20:] = 0
    t = torch.tensor([5, 150])
    cond = torch.randn(B, S, d, generator=gen)
    R = torch.randn(B, L, V, generator=gen)
    monkeypatch.setattr(rt, "next_seed", lambda: 777)
    with rt.use_precision(prec):
        dec = make_decoder(V, d, H, NL, FF, dropout=0.1)
        dec.train()
        logits = dec(xt.to(dev), t.to(dev), cond.to(dev))
        (logits * R.to(dev)).sum().backward()
    sd = {n: p.detach().cpu().clone().requires_grad_(True) for n, p in dec.named_parameters()}
    ref = O.decoder_forward(sd, xt, t, cond, None, H=H, num_layers=NL, dropout=0.1, seed=777)
    (ref * R).sum().backward()
    close(logits, ref.detach(), rtol=tol, what=f"{prec} logits")
    for n in ("blocks.0.self_attn.in_proj_weight", "blocks.1.ff.0.weight", "head.weight", "tok_emb.weight",
              "blocks.0.norm2.weight", "blocks.1.film_layer.scale_proj.weight", "time_proj.weight"):
        p = dict(dec.named_parameters())[n]
        close(p.grad, sd[n].grad, rtol=(3 * tol), atol=1e-6, what=f"{prec} grad {n}")


def _encoder(geom, d_model):
    from models.acoustic_encoder import AcousticEncoder
    over = {k: v for k, v in geom.items()}
    enc = AcousticEncoder(wavlm_name=over, d_model=d_model)
    sd = enc.state_dict()
    for n, v in wavlm_sd(O.wavlm_geometry(**geom), d_model).items():
        assert n in sd, n
        sd[n] = v
    enc.load_state_dict(sd)
    return enc.to(dev).eval()


def test_wavlm_small_fp32_matches_reference():
    g = load("wavlm")
    rt = _rt()
    with rt.use_precision("fp32"):
        enc = _encoder(SMALL_WAVLM, 64)
        feats, m, pooled = enc(T(g["small_wave"]).to(dev))
    assert m is None and pooled is None
    close(feats, g["small_feats"], rtol=1e-4, what="small wavlm feats")


@pytest.mark.parametrize("prec,tol", [("fp32", 1e-4), ("bf16", 5e-2)])
def test_wavlm_base_matches_reference(prec, tol):
    g = load("wavlm")
    rt = _rt()
    with rt.use_precision(prec):
        enc = _encoder({}, 512)
        feats, _, _ = enc(T(g["base_wave"]).to(dev))
    close(feats.float(), g["base_feats"], rtol=tol, what=f"{prec} base wavlm feats")


def test_wavlm_base_10s_batch_matches_oracle_bf16():
    """C2 geometry (10 s -> S=499) on 2 utterances: bf16 kernels vs fp32 oracle."""
    rt = _rt()
    gen = torch.Generator().manual_seed(9)
    wave = 0.1 * torch.randn(2, 160000, generator=gen)
    with rt.use_precision("bf16"):
        enc = _encoder({}, 512)
        feats, _, _ = enc(wave.to(dev))
    assert feats.shape == (2, 499, 512)
    sd = wavlm_sd(O.wavlm_geometry(), 512)
    ref = O.acoustic_encoder(sd, wave, O.wavlm_geometry(), 512)
    close(feats.float(), ref, rtol=5e-2, what="10 s bf16 encoder")


@pytest.mark.parametrize("tag,geom,V,d,H,NL,FF,Tn", [
    ("step_c1", {}, 8000, 128, 2, 2, 2048, 10),
    ("step_repeat", SMALL_WAVLM, 500, 128, 2, 1, 256, 20),
])
def test_train_step_fp32_matches_reference(tag, geom, V, d, H, NL, FF, Tn, monkeypatch):
    """Four teacher-forced steps of train_one_epoch (incl. one L_fd step) vs the reference fixture."""
    import train as T_
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from fddm_hip.optim import FusedAdamW
    from models.projection import SpeechProjector, TextEmbedding, TextProjector
    g = load(tag)
    rt = _rt()
    with rt.use_precision("fp32"):
        enc = _encoder(geom, d)
        dec = make_decoder(V, d, H, NL, FF)
        sp, te, tp = SpeechProjector(d, 256), TextEmbedding(V, 256), TextProjector(256, 256)
        params = _step_params(V, d, NL, FF, H)
        for pre, m in (("s_proj.", sp), ("t_embed.", te), ("t_proj.", tp)):
            m.load_state_dict({n: params[pre + n] for n, _ in m.named_parameters()})
            m.to(dev)
        xts = [T(x).to(dev) for x in g["xts"]]
        ts = iter([T(x).to(dev) for x in g["ts"]])
        rec = {"kl": [], "lfd": []}

        class TF(T_.SchedulerAdapter):
            i = 0

            def sample_q(self, x0, t):
                v = xts[TF.i]
                TF.i += 1
                return v

            def kl_term(self, *a, **k):
                v = super().kl_term(*a, **k)
                rec["kl"].append(v)
                return v

        orig = T_.lfd_loss

        def rl(*a, **k):
            v = orig(*a, **k)
            rec["lfd"].append(v)
            return v

        monkeypatch.setattr(T_, "lfd_loss", rl)
        trainable = list(dec.parameters()) + list(sp.parameters()) + list(te.parameters()) + list(tp.parameters())
        opt = FusedAdamW(trainable, lr=2e-4, weight_decay=0.01)
        cfg = T_.Config(seed=1, data={"pad_id": 0}, model={}, diffusion={"T": Tn}, inference={}, optim={},
                        lfd={"n_step_fd": 4, "tau": 1.0, "lambda_offdiag": 5e-3}, log={"log_every": 1000})
        sch = TF(DiscreteDiffusionScheduler(K=V, T=Tn, device=dev))
        loader = [(T(w), T(x)) for w, x in zip(g["waves"], g["x0s"])]
        init = {("decoder." + n): p.detach().cpu().clone() for n, p in dec.named_parameters()}
        init.update({k: v.clone() for k, v in params.items() if not k.startswith("decoder.")})
        T_.train_one_epoch(enc, dec, sp, te, tp, sch, loader, opt, dev, cfg, 1, None, 1, False,
                           draw_t=lambda B: next(ts))
    close(torch.stack([v.detach().cpu() for v in rec["kl"]]), g["kl"], rtol=1e-4, what="per-step KL")
    close(torch.stack([v.detach().cpu() for v in rec["lfd"]]), g["lfd"], rtol=1e-4, what="L_fd")
    final = {("decoder." + n): p.detach().cpu() for n, p in dec.named_parameters()}
    for pre, m in (("s_proj.", sp), ("t_embed.", te), ("t_proj.", tp)):
        final.update({pre + n: p.detach().cpu() for n, p in m.named_parameters()})
    noise_only = ("s_proj.proj.net.0.bias", "t_proj.proj.net.0.bias")
    for n, p in final.items():
        if n in noise_only:
            continue
        dp = p.double() - init[n].double()
        close((dp ** 2).sum(), g["dp_sq." + n], rtol=5e-3, atol=1e-12, what="update " + n)
        if "p." + n in g and "in_proj_bias" not in n:
            err = (p.double() - T(g["p." + n]).double()).abs()
            assert (err > 4e-6).float().mean().item() < 0.02, n


@pytest.mark.parametrize("with_lfd", [False, True])
def test_bf16_kl_gradient_handover_matches_fp32_gradient_path(with_lfd):
    """bf16 mode hands the KL's logits gradient to the head backward in bf16 (functions.KLFn / HeadFn);
    the decoder gradients must equal those of the plain path (fp32 dlogits through autograd, cast in the
    head backward) — alone and summed with an L_fd-style second consumer of the logits."""
    from fddm_hip import functions as FN
    from fddm_hip import runtime as rt_
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    import train as T_
    gen = torch.Generator().manual_seed(5)
    V, d, B, L, S = 1000, 128, 2, 16, 20
    xt = torch.randint(1, V, (B, L), generator=gen).to(dev)
    x0 = torch.randint(1, V, (B, L), generator=gen).to(dev)
    t = torch.tensor([3, 7]).to(dev)
    cond = torch.randn(B, S, d, generator=gen).to(dev)
    R = torch.randn(B, L, V, generator=gen).to(dev)
    sch = T_.SchedulerAdapter(DiscreteDiffusionScheduler(K=V, T=10, device=dev))
    grads = []
    for handover in (True, False):
        with rt_.use_precision("bf16"):
            dec = make_decoder(V, d, 2, 2, 256)
            dec.train()
            if not handover:
                saved = FN._head_outputs
                FN._head_outputs = type("NoReg", (dict,), {"__setitem__": lambda self, k, v: None})()
            try:
                logits = dec(xt, t, cond)
                loss = sch.kl_term(xt, x0, logits, t)
                if with_lfd:
                    loss = loss + 1e-3 * (logits * R).sum()
                loss.backward()
            finally:
                if not handover:
                    FN._head_outputs = saved
            grads.append({n: p.grad.detach().clone() for n, p in dec.named_parameters() if p.grad is not None})
    assert grads[0].keys() == grads[1].keys()
    for n in grads[0]:
        close(grads[0][n], grads[1][n], rtol=2e-2, atol=1e-6, what=n)
    assert any(g.abs().max().item() > 0 for g in grads[0].values())


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("geom,d", [(SMALL_WAVLM, 128), ({}, 768), ({}, 512)])
def test_graphed_encoder_slots_match_eager(prec, geom, d):
    """train._encoded's HIP-graph replay of the frozen encoder (fddm_hip/graphs.py: two slots, a private memory pool
    each) yields, for every batch, the eager forward's features — at the yield and still after main-stream work
    that allocates and writes memory while the next batch is encoded on the side stream (a shared pool let slot 0's
    replay overwrite slot 1's output; the split-K memset node raced the GEMM on replays). bf16: bit-identical;
    fp32: within 1e-5 of the feature scale (split-K f32 atomics sum in launch order)."""
    import train as T_
    rt = _rt()

    class Opt:
        param_groups = [{"params": []}]

    with rt.use_precision(prec):
        enc = _encoder(geom, d)
        gen = torch.Generator().manual_seed(3)
        sec = 1 if geom else 4
        loader = [(0.1 * torch.randn(2, 16000 * sec, generator=gen), torch.zeros(2, 8, dtype=torch.long))
                  for _ in range(5)]
        got = []
        for c, _, _ in T_._encoded(enc, loader, dev, Opt()):
            a = c.float().clone()
            junk = [torch.randn(2048, 2048, device=dev) for _ in range(3)]
            for _ in range(3):
                junk[0] = junk[1] @ junk[2] + junk[0]
            del junk
            got.append((a, c.float().clone()))
        torch.cuda.synchronize()
        refs = [enc(w.to(dev))[0].float() for w, _ in loader]
    for i, ((a, b), r) in enumerate(zip(got, refs)):
        tol = 0.0 if prec == "bf16" else 1e-5 * float(r.abs().max())
        assert float((a - r).abs().max()) <= tol, f"batch {i} at yield"
        assert float((b - r).abs().max()) <= tol, f"batch {i} after main-stream work"


def test_graphed_encoder_recaptures_after_weight_change():
    """Changing a frozen encoder's parameters in place (or its projection) between replays: the graph runner sees
    the re-prepared weights and recaptures, so replays follow the new weights (no stale or freed buffers)."""
    from fddm_hip.graphs import GraphedEncoder
    rt = _rt()
    with rt.use_precision("bf16"):
        enc = _encoder(SMALL_WAVLM, 96)
        assert enc.use_proj
        ge = GraphedEncoder(enc)
        w = 0.1 * torch.randn(2, 16000, generator=torch.Generator().manual_seed(5)).to(dev)
        first = ge.run(w, 0).float().clone()
        with torch.no_grad():
            enc.backbone.encoder.layers[0].feed_forward.output_dense.weight.mul_(1.5)
            enc.proj.weight.add_(0.01)
        again = ge.run(w, 0).float().clone()
        ref = enc(w)[0].float()
        torch.cuda.synchronize()
    assert float((again - ref).abs().max()) == 0.0
    assert float((again - first).abs().max()) > 0.0


def test_graphed_encoder_survives_clear_cache():
    """rt.clear_cache() (load_checkpoint calls it) drops the runtime's cached relative-bias table and bf16 encoder.proj
    weight that a captured encoder graph reads by address: the graph runner holds those buffers for its
    captures and recaptures on the next run, so a replay after the clear equals the eager forward."""
    from fddm_hip.graphs import GraphedEncoder
    rt = _rt()
    with rt.use_precision("bf16"):
        enc = _encoder(SMALL_WAVLM, 96)
        assert enc.use_proj
        ge = GraphedEncoder(enc)
        w = 0.1 * torch.randn(2, 16000, generator=torch.Generator().manual_seed(6)).to(dev)
        first = ge.run(w, 1).float().clone()
        slot = ge.cache[next(iter(ge.cache))][1]
        assert len(slot.keep) >= 2, "the capture must hold the cached tensors it reads"
        rt.clear_cache()
        junk = [torch.randn(1024, 1024, device=dev) for _ in range(8)]     # reuse the freed cache memory
        for j in junk:
            j.mul_(3.0)
        again = ge.run(w, 1).float().clone()
        ref = enc(w)[0].float()
        torch.cuda.synchronize()
    assert float((again - ref).abs().max()) == 0.0
    assert float((first - ref).abs().max()) == 0.0


@pytest.mark.parametrize("prec,tol", [("fp32", 1e-4), ("bf16", 3e-2)])
def test_train_step_odd_vocab_matches_oracle(prec, tol, monkeypatch):
    """A vocabulary the one-pass KL kernel is not built for (V = 997: V % 4 != 0) and the bf16 softmax-backward
    hand-over skips (V % 8 != 0): two teacher-forced train_one_epoch steps (a KL step and an L_fd step) take the
    two-pass KL and the f32 softmax backward, and match oracle_train_step from the same condition."""
    import torch.nn as nn

    import train as T_
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from fddm_hip.optim import FusedAdamW
    from models.projection import SpeechProjector, TextEmbedding, TextProjector
    rt = _rt()
    V, d, H, NL, FF, B, L, S, Tn = 997, 128, 2, 2, 256, 3, 24, 30, 20

    class Identity(nn.Module):      # the "encoder": the loader hands the acoustic condition itself
        def forward(self, c):
            return c, None, None

    gen = torch.Generator().manual_seed(12)
    conds = [torch.randn(B, S, d, generator=gen) for _ in range(2)]
    x0s = [torch.randint(1, V, (B, L), generator=gen) for _ in range(2)]
    x0s[0][1, 17:] = 0
    ts = [torch.tensor([1, 9, 20]), torch.tensor([4, 2, 13])]
    betas, ab = O.sched_tables(Tn)
    xts = [O.sample_xt(x0, t, V, ab, seed=5 + i) for i, (x0, t) in enumerate(zip(x0s, ts))]
    params = _step_params(V, d, NL, FF, H)
    rec = {"kl": [], "lfd": []}
    with rt.use_precision(prec):
        dec = make_decoder(V, d, H, NL, FF)
        sp, te, tp = SpeechProjector(d, 256), TextEmbedding(V, 256), TextProjector(256, 256)
        for pre, m in (("s_proj.", sp), ("t_embed.", te), ("t_proj.", tp)):
            m.load_state_dict({n: params[pre + n] for n, _ in m.named_parameters()})
            m.to(dev)
        xq = iter([x.to(dev) for x in xts])
        tq = iter([t.to(dev) for t in ts])

        class TF(T_.SchedulerAdapter):
            def sample_q(self, x0, t):
                return next(xq)

            def kl_term(self, *a, **k):
                v = super().kl_term(*a, **k)
                rec["kl"].append(float(v.detach()))
                return v

        orig = T_.lfd_loss

        def rl(*a, **k):
            v = orig(*a, **k)
            rec["lfd"].append(float(v.detach()))
            return v

        monkeypatch.setattr(T_, "lfd_loss", rl)
        trainable = list(dec.parameters()) + list(sp.parameters()) + list(te.parameters()) + list(tp.parameters())
        opt = FusedAdamW(trainable, lr=2e-4, weight_decay=0.01)
        cfg = T_.Config(seed=1, data={"pad_id": 0}, model={}, diffusion={"T": Tn}, inference={}, optim={},
                        lfd={"n_step_fd": 4, "tau": 1.0, "lambda_offdiag": 5e-3}, log={"log_every": 1000})
        loader = list(zip(conds, x0s))
        T_.train_one_epoch(Identity(), dec, sp, te, tp, TF(DiscreteDiffusionScheduler(K=V, T=Tn, device=dev)), loader,
                           opt, dev, cfg, 3, None, 1, False, draw_t=lambda B_: next(tq))
        torch.cuda.synchronize()
    ocfg = dict(d_model=d, nhead=H, num_layers=NL, pad_id=0, n_step_fd=4, tau=1.0, lambda_offdiag=5e-3)
    oopt = O.OracleAdamW()
    ref = [O.oracle_train_step(params, None, None, None, x0s[i], ts[i], xts[i], ocfg, oopt, 3 + i, betas, ab,
                               c=conds[i]) for i in range(2)]
    close(torch.tensor(rec["kl"]), torch.tensor([r["kl"] for r in ref]), rtol=tol, what=f"{prec} odd-V KL")
    close(torch.tensor(rec["lfd"]), torch.tensor([ref[1]["lfd"]]), rtol=tol, what=f"{prec} odd-V L_fd")
    final = {("decoder." + n): p.detach().cpu() for n, p in dec.named_parameters()}
    for pre, m in (("s_proj.", sp), ("t_embed.", te), ("t_proj.", tp)):
        final.update({pre + n: p.detach().cpu() for n, p in m.named_parameters()})
    init = _step_params(V, d, NL, FF, H)
    for n in ("decoder.head.weight", "decoder.head.bias", "decoder.blocks.0.ff.0.weight", "t_embed.proj.weight"):
        # update norms (AdamW's first steps move near-zero-gradient elements by ~lr in a direction rounding picks)
        got = float(((final[n].double() - init[n].double()) ** 2).sum())
        want = float(((params[n].double() - init[n].double()) ** 2).sum())
        assert abs(got - want) <= (5e-3 if prec == "fp32" else 5e-2) * want, f"{prec} odd-V update {n}: {got} vs {want}"
