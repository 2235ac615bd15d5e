"""Generate the golden fixtures in tests/golden/*.npz by running the REFERENCE code in this container.

Run from the repo root:  python tests/golden/make_golden.py
The reference is imported read-only from /root/reference (bytecode writing disabled). Only small
input/output arrays are saved; the reference itself never leaves this container. WavLM weights are not
downloadable offline, so `WavLMModel.from_pretrained` is replaced by a local constructor that builds
`WavLMModel(WavLMConfig(**geometry))` and loads numpy-PCG64 weights (oracle/weights.py), exactly as the
tests rebuild them on the GPU box.
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
REF = os.environ.get("FDDM_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.set_num_threads(8)
from oracle.weights import load_pcg, pcg_state_dict  # noqa: E402

OUT = HERE
C = {}  # name -> dict of arrays


def save(name, **arrs):
    arrs = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in arrs.items()}
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrs)
    print("wrote", name, {k: v.shape for k, v in arrs.items()})


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


# ----------------------------------------------------------------------------------------------
def gen_sched():
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler

    out = {}
    for K, T in [(8000, 10), (8000, 200), (2000, 200)]:
        s = DiscreteDiffusionScheduler(K=K, T=T, device=torch.device("cpu"), beta_max=0.2)
        out[f"betas_{K}_{T}"] = s.betas
        out[f"alpha_bar_{K}_{T}"] = s.alpha_bar
        # q_sample: one row per t with x0 = 10 (as in scripts/sanity_check_scheduler.py)
        ts = torch.arange(1, T + 1)
        x0 = torch.zeros(T, 1, K)
        x0[:, 0, 10] = 1.0
        p = s.q_sample(x0, ts)[:, 0, :]
        out[f"qs_hi_{K}_{T}"] = p[:, 10]
        out[f"qs_lo_{K}_{T}"] = p[:, 11]
        out[f"qs_rowsum_{K}_{T}"] = p.sum(-1)
        # q_posterior on a perturbed x0hat, row sums (sanity_check_scheduler.py:22-26)
        g = torch.Generator().manual_seed(7)
        x0hat = torch.softmax(torch.randn(T, 1, K, generator=g), -1)
        post = s.q_posterior(p[:, None, :], x0hat, ts)
        out[f"qpost_rowsum_{K}_{T}"] = post[:, 0, :].sum(-1)
        out[f"qpost_row_{K}_{T}"] = post[:, 0, :16]
    save("sched", **out)


def gen_kl():
    import train as ref_train
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler

    B, L, V, T = 3, 8, 2000, 200
    r = rng(11)
    s = DiscreteDiffusionScheduler(K=V, T=T, device=torch.device("cpu"), beta_max=0.2)
    ad = ref_train.SchedulerAdapter(s)
    t = torch.tensor([1, 100, 200])
    x0 = torch.from_numpy(r.integers(1, V, size=(B, L))).long()
    x0[0, 6:] = 0
    x0[2, 7:] = 0
    xt = torch.from_numpy(r.integers(0, V, size=(B, L))).long()
    keep = torch.from_numpy(r.random((B, L)) < 0.5)
    xt = torch.where(keep, x0, xt)
    logits = torch.from_numpy(2.0 * r.standard_normal((B, L, V), dtype=np.float32))
    logits[1, 3, xt[1, 3]] += 6.0
    x_mask = x0 != 0
    lg = logits.clone().requires_grad_(True)
    kl = ad.kl_term(xt, x0, lg, t, x_mask)
    kl.backward()
    lg2 = logits.clone().requires_grad_(True)
    kl2 = ad.kl_term(xt, x0, lg2, t, None)
    kl2.backward()
    wt = ad.w_t(t)
    save("kl", t=t, x0=x0, xt=xt, logits=logits, x_mask=x_mask, kl=kl, dlogits=lg.grad,
         kl_nomask=kl2, dlogits_nomask=lg2.grad, w_t=wt, betas=s.betas)


def gen_rope():
    from models.denoise_decoder import RoPEEmbedding

    out = {}
    r = rng(12)
    for d, L in [(8, 5), (128, 7), (512, 9)]:
        pe = RoPEEmbedding(d)
        cos, sin = pe(L, torch.device("cpu"))
        x = torch.from_numpy(r.standard_normal((2, L, d), dtype=np.float32))
        out[f"x_{d}"] = x
        out[f"y_{d}"] = RoPEEmbedding.apply_rotary_pos_emb(x, cos, sin)
        out[f"inv_freq_{d}"] = pe.inv_freq
    save("rope", **out)


def gen_lfd():
    from losses.fddm_losses import lfd_loss

    r = rng(13)
    za = torch.from_numpy(r.standard_normal((4, 16, 32), dtype=np.float32)).requires_grad_(True)
    zb = torch.from_numpy((0.5 * za.detach().numpy() + r.standard_normal((4, 16, 32), dtype=np.float32))).requires_grad_(True)
    loss = lfd_loss(za, zb, lambda_offdiag=5e-3)
    loss.backward()
    save("lfd", za=za.detach(), zb=zb.detach(), loss=loss, dza=za.grad, dzb=zb.grad)


def _dec_grads_subset(model):
    out = {}
    for n, p in model.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        out["g_sum." + n] = g.sum()
        out["g_sq." + n] = (g.double() ** 2).sum()
        if g.numel() <= 70000:
            out["g." + n] = g
    return out


def gen_decoder():
    from models.denoise_decoder import DenoisingTransformerDecoder

    V, d, H, NL, FF = 1000, 128, 2, 2, 256
    B, L, S = 2, 16, 20
    r = rng(14)
    dec = DenoisingTransformerDecoder(vocab_size=V, d_model=d, nhead=H, num_layers=NL, dim_ff=FF,
                                      dropout=0.0, max_len=1024, pad_id=0)
    load_pcg(dec, prefix="dec.", pad_row=("tok_emb.weight", 0))
    dec.train()
    xt = torch.from_numpy(r.integers(1, V, size=(B, L))).long()
    xt[1, 12:] = 0
    x_mask = torch.ones(B, L, dtype=torch.bool)
    x_mask[1, 11:] = False
    t = torch.tensor([3, 170])
    cond = torch.from_numpy(r.standard_normal((B, S, d), dtype=np.float32)).requires_grad_(True)
    R = torch.from_numpy(r.standard_normal((B, L, V), dtype=np.float32))
    logits = dec(xt, t, cond, x_mask=x_mask, c_mask=None)
    (logits * R).sum().backward()
    out = dict(xt=xt, x_mask=x_mask, t=t, cond=cond.detach(), R=R, logits=logits.detach(), dcond=cond.grad)
    out.update(_dec_grads_subset(dec))
    # default-mask path (x_mask=None -> xt != pad) forward only
    with torch.no_grad():
        out["logits_defmask"] = dec(xt, t, cond.detach())
    save("decoder", **out)


# ---------------------------------------------------------------- WavLM (local stand-in for hub)
SMALL_WAVLM = dict(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=256,
                   conv_dim=(32,) * 7, num_conv_pos_embedding_groups=4)


def _patch_from_pretrained(geometry: dict, prefix: str):
    from transformers import WavLMConfig, WavLMModel
    import models.acoustic_encoder as ae

    def fake_from_pretrained(name, *a, **k):
        m = WavLMModel(WavLMConfig(**geometry))
        load_pcg(m, prefix=prefix)
        return m

    ae.WavLMModel.from_pretrained = staticmethod(fake_from_pretrained)


def gen_wavlm():
    from models.acoustic_encoder import AcousticEncoder

    r = rng(15)
    out = {}
    # small geometry, 2 utterances x 1 s, proj 128 -> 64
    _patch_from_pretrained(SMALL_WAVLM, "backbone.")
    enc = AcousticEncoder(wavlm_name="local-small", d_model=64)
    load_pcg(enc, prefix="")  # PCG on the full encoder names (backbone.* and proj.*)
    enc.eval()
    wave = torch.from_numpy(0.1 * r.standard_normal((2, 16000), dtype=np.float32))
    with torch.no_grad():
        feats, fm, pooled = enc(wave)
        hid = enc.backbone(wave).last_hidden_state
        fe = enc.backbone.feature_extractor(wave)
    out.update(small_wave=wave, small_feats=feats, small_hidden=hid, small_fe=fe)
    # base geometry (WavLMConfig() defaults), 1 utterance x 1 s, proj 768 -> 512
    _patch_from_pretrained({}, "backbone.")
    enc = AcousticEncoder(wavlm_name="local-base", d_model=512)
    load_pcg(enc, prefix="")
    enc.eval()
    wave = torch.from_numpy(0.1 * r.standard_normal((1, 16000), dtype=np.float32))
    with torch.no_grad():
        feats, _, _ = enc(wave)
        fe = enc.backbone.feature_extractor(wave)
    out.update(base_wave=wave, base_feats=feats, base_fe_sum=fe.sum(), base_fe_sq=(fe.double() ** 2).sum(),
               base_fe_slice=fe[0, :8, :64])
    save("wavlm", **out)


# ---------------------------------------------------------------- full training step (train.py)
def gen_step(tag, geometry, B, L, V, d, H, NL, FF, T, nsteps, seconds=1):
    import train as ref_train
    from models.acoustic_encoder import AcousticEncoder
    from models.denoise_decoder import DenoisingTransformerDecoder
    from models.projection import SpeechProjector, TextEmbedding, TextProjector
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler

    r = rng(16)
    _patch_from_pretrained(geometry, "backbone.")
    enc = AcousticEncoder(wavlm_name="local", d_model=d)
    load_pcg(enc, prefix="")
    dec = DenoisingTransformerDecoder(vocab_size=V, d_model=d, nhead=H, num_layers=NL, dim_ff=FF,
                                      dropout=0.0, max_len=1024, pad_id=0)
    load_pcg(dec, prefix="dec.", pad_row=("tok_emb.weight", 0))
    s_proj = SpeechProjector(d_in=d, d_proj=256)
    t_embed = TextEmbedding(vocab=V, d_out=256, mode="logits")
    t_proj = TextProjector(d_in=256, d_proj=256)
    load_pcg(s_proj, prefix="s_proj.")
    load_pcg(t_embed, prefix="t_embed.")
    load_pcg(t_proj, prefix="t_proj.")
    init_params = {}
    for pre, m in [("decoder.", dec), ("s_proj.", s_proj), ("t_embed.", t_embed), ("t_proj.", t_proj)]:
        for n, p in m.named_parameters():
            init_params[pre + n] = p.detach().clone()

    sch = DiscreteDiffusionScheduler(K=V, T=T, device=torch.device("cpu"), beta_max=0.2)
    waves, x0s, ts, xts = [], [], [], []
    for i in range(nsteps):
        w = torch.from_numpy(0.1 * r.standard_normal((B, 16000 * seconds), dtype=np.float32))
        x0 = torch.from_numpy(r.integers(1, V, size=(B, L))).long()
        for b in range(B):
            ell = int(r.integers(L // 2, L + 1))
            x0[b, ell:] = 0
        t = torch.from_numpy(r.integers(1, T + 1, size=(B,))).long()
        keep = torch.from_numpy(r.random((B, L)) < 0.6)
        xt = torch.where(keep, x0, torch.from_numpy(r.integers(0, V, size=(B, L))).long())
        waves.append(w); x0s.append(x0); ts.append(t); xts.append(xt)

    rec = {"kl": [], "lfd": [], "c_step1": None, "logits_step1": None}

    class TFAdapter(ref_train.SchedulerAdapter):
        i = 0

        def sample_q(self, x0, t):
            return xts[TFAdapter.i]

        def kl_term(self, xt, x0, logits_x0, t, x_mask=None):
            v = super().kl_term(xt, x0, logits_x0, t, x_mask)
            rec["kl"].append(float(v.item()))
            if TFAdapter.i == 0:
                rec["logits_step1"] = logits_x0.detach().clone()
            TFAdapter.i += 1
            return v

    orig_lfd = ref_train.lfd_loss

    def rec_lfd(za, zb, lambda_offdiag=5e-3):
        v = orig_lfd(za, zb, lambda_offdiag=lambda_offdiag)
        rec["lfd"].append(float(v.item()))
        return v

    orig_randint = torch.randint
    t_iter = iter(ts)

    def tf_randint(low, high, size, *a, **k):
        if low == 1 and high == T + 1:
            return next(t_iter).clone()
        return orig_randint(low, high, size, *a, **k)

    orig_enc_fwd = enc.forward

    def rec_enc(w, lengths=None):
        o = orig_enc_fwd(w, lengths)
        if rec["c_step1"] is None:
            rec["c_step1"] = o[0].detach().clone()
        return o

    enc.forward = rec_enc
    params = list(dec.parameters()) + list(s_proj.parameters()) + list(t_embed.parameters()) + list(t_proj.parameters())
    optim = torch.optim.AdamW(params, lr=2e-4, weight_decay=0.01)
    cfg = ref_train.Config(seed=1337, data={"pad_id": 0}, model={}, diffusion={"T": T}, inference={},
                           optim={}, lfd={"n_step_fd": 4, "tau": 1.0, "lambda_offdiag": 5e-3},
                           log={"log_every": 50})
    loader = list(zip(waves, x0s))
    ref_train.lfd_loss = rec_lfd
    torch.randint = tf_randint
    try:
        gs, avg = ref_train.train_one_epoch(enc, dec, s_proj, t_embed, t_proj, TFAdapter(sch), loader, optim,
                                            torch.device("cpu"), cfg, 1, None, 1, False)
    finally:
        torch.randint = orig_randint
        ref_train.lfd_loss = orig_lfd
    out = dict(waves=torch.stack(waves), x0s=torch.stack(x0s), ts=torch.stack(ts), xts=torch.stack(xts),
               kl=np.array(rec["kl"]), lfd=np.array(rec["lfd"]), avg_loss=np.array(avg),
               c_step1=rec["c_step1"], logits1_sum=rec["logits_step1"].sum(),
               logits1_sq=(rec["logits_step1"].double() ** 2).sum(), logits1_slice=rec["logits_step1"][:, :4, :64])
    wt = torch.stack([sch.alpha_bar[t - 1].mean() for t in ts])
    out["w_t_mean"] = wt
    for pre, m in [("decoder.", dec), ("s_proj.", s_proj), ("t_embed.", t_embed), ("t_proj.", t_proj)]:
        for n, p in m.named_parameters():
            key = pre + n
            dp = (p.detach().double() - init_params[key].double())
            out["p_sum." + key] = p.detach().double().sum()
            out["dp_sum." + key] = dp.sum()
            out["dp_sq." + key] = (dp ** 2).sum()
            if p.numel() <= 20000:
                out["p." + key] = p.detach()
    save(tag, **out)


# ---------------------------------------------------------------- jumpy sampler (C5)
def jumpy_case_inputs(i, B, L, K):
    """Seeded inputs of posterior case i (regenerated by tests/test_oracle_golden.py; numpy PCG64 is
    platform-independent), so the fixture stores only the outputs."""
    r = rng(300 + i)
    logits = torch.from_numpy(3.0 * r.standard_normal((B, L, K), dtype=np.float32))
    xt = torch.from_numpy(r.integers(0, K, size=(B, L))).long()
    # make x_t a serious contender on some rows
    boost = torch.from_numpy(r.uniform(-10.0, 6.0, size=(B, L)).astype(np.float32))
    logits.scatter_add_(-1, xt[..., None], boost[..., None])
    return logits, xt


def gen_jumpy():
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from models.denoise_decoder import DenoisingTransformerDecoder
    import sampler.jumpy_sampler as js

    out = {}
    r = rng(21)
    # A. exact multi-step posterior argmax for given logits (q_posterior_multi_step + argmax)
    K, T = 2000, 200
    sch = DiscreteDiffusionScheduler(K=K, T=T, device=torch.device("cpu"), beta_max=0.2)
    cases = [([20, 20, 20, 20], 5), ([5, 5, 5, 5], 5), ([1, 1, 1, 1], 1), ([200, 150, 90, 7], 5),
             ([10, 12, 3, 40], 2), ([2, 30, 100, 199], 1)]
    B, L = 4, 48
    for i, (ts, delta) in enumerate(cases):
        t = torch.tensor(ts)
        logits, xt = jumpy_case_inputs(i, B, L, K)
        p = torch.softmax(logits, -1)
        oh = torch.zeros(B, L, K)
        oh.scatter_(-1, xt[..., None], 1.0)
        post = sch.q_posterior_multi_step(oh, p, t, delta)
        out[f"c{i}_t"] = t
        out[f"c{i}_delta"] = np.int64(delta)
        out[f"c{i}_xt"] = xt
        out[f"c{i}_next"] = post.argmax(-1)
        out[f"c{i}_post_max"] = post.max(-1).values
    # B. full sampler run (exact, greedy) with a small decoder, x_T drawn from torch.manual_seed(5)
    V, d, H, NL, FF = 1000, 128, 2, 2, 256
    Bs, S, Ls = 3, 20, 16
    dec = DenoisingTransformerDecoder(vocab_size=V, d_model=d, nhead=H, num_layers=NL, dim_ff=FF, dropout=0.1,
                                      max_len=1024, pad_id=0)
    load_pcg(dec, prefix="dec.", pad_row=("tok_emb.weight", 0))
    dec.eval()
    cond = torch.from_numpy(r.standard_normal((Bs, S, d), dtype=np.float32))
    sch2 = DiscreteDiffusionScheduler(K=V, T=200, device=torch.device("cpu"), beta_max=0.2)
    for mode in ("exact", "fast"):
        smp = js.DiffusionJumpySampler(sch2, dec, K=V, T_train=200, T_infer=20, r=5, greedy=True,
                                       posterior_mode="map", sampling_mode=mode, device=torch.device("cpu"))
        seq = []
        orig = smp._jump_once

        def rec(x, t_scalar, delta, cond_c, seq_len, _orig=orig, _seq=seq):
            nx, p = _orig(x, t_scalar=t_scalar, delta=delta, cond_c=cond_c, seq_len=seq_len)
            _seq.append((x.clone(), t_scalar, delta, nx.clone(), p.argmax(-1)))
            return nx, p

        smp._jump_once = rec
        torch.manual_seed(5)
        with torch.no_grad():
            x0, plast = smp.sample(cond, seq_len=Ls)
        out[f"run_{mode}_xT"] = seq[0][0]
        out[f"run_{mode}_ts"] = np.array([s_[1] for s_ in seq])
        out[f"run_{mode}_deltas"] = np.array([s_[2] for s_ in seq])
        out[f"run_{mode}_xs"] = torch.stack([s_[3] for s_ in seq])
        out[f"run_{mode}_x0hat"] = torch.stack([s_[4] for s_ in seq])
        out[f"run_{mode}_x0"] = x0
        out[f"run_{mode}_plast_max"] = plast.max(-1).values
    out["run_cond"] = cond
    save("jumpy", **out)


# ---------------------------------------------------------------- CER / WER evaluation
def gen_cer():
    from models.evaluate import _ids_to_text_one, calculate_cer, calculate_wer

    r = rng(31)
    pool = list("我這可以交流道台有一沒中在大個們公路臺捷運新高什麼自己你是的人就問題還雄但他知政府現也") + [" "] * 6
    refs, hyps = [], []
    for i in range(60):
        n = int(r.integers(0, 40)) if i % 10 else 0
        ref = "".join(r.choice(pool, size=n))
        hyp = list(ref)
        for _ in range(int(r.integers(0, 8))):          # random edits
            op = int(r.integers(0, 3))
            pos = int(r.integers(0, len(hyp) + 1))
            if op == 0 and hyp and pos < len(hyp):
                hyp[pos] = str(r.choice(pool))
            elif op == 1:
                hyp.insert(pos, str(r.choice(pool)))
            elif hyp and pos < len(hyp):
                del hyp[pos]
        hyp = "".join(hyp) if i % 13 else ""
        refs.append(ref)
        hyps.append(hyp)
    cer = [calculate_cer(a, b) for a, b in zip(refs, hyps)]
    wer = [calculate_wer(a, b) for a, b in zip(refs, hyps)]

    class Rec:  # records the ids _ids_to_text_one hands to the tokenizer
        def DecodeIds(self, ids):
            return ",".join(str(i) for i in ids)

    ids = torch.from_numpy(r.integers(0, 12, size=(40, 24))).long()
    clean = [_ids_to_text_one(ids[i], Rec(), pad_id=0, bos_id=1 if i % 2 else None, eos_id=2 if i % 3 else None)
             for i in range(40)]
    save("cer", refs=np.array(refs), hyps=np.array(hyps), cer=np.array(cer), wer=np.array(wer), ids=ids,
         clean=np.array(clean))


if __name__ == "__main__":
    which = sys.argv[1:] or ["sched", "kl", "rope", "lfd", "decoder", "wavlm", "step_c1", "step_repeat", "jumpy", "cer"]
    if "sched" in which:
        gen_sched()
    if "kl" in which:
        gen_kl()
    if "rope" in which:
        gen_rope()
    if "lfd" in which:
        gen_lfd()
    if "decoder" in which:
        gen_decoder()
    if "wavlm" in which:
        gen_wavlm()
    if "step_c1" in which:
        # C1: WavLM-base, 2-layer d=128 decoder (H=2 -> head_dim 64), 4 x (1 s, 32 tokens), T=10, V=8000
        gen_step("step_c1", {}, B=4, L=32, V=8000, d=128, H=2, NL=2, FF=2048, T=10, nsteps=4)
    if "jumpy" in which:
        gen_jumpy()
    if "cer" in which:
        gen_cer()
    if "step_repeat" in which:
        # S (49) < L (64): exercises the repeat-last-frame alignment branch (train.py:385-387)
        gen_step("step_repeat", SMALL_WAVLM, B=3, L=64, V=500, d=128, H=2, NL=1, FF=256, T=20, nsteps=4)
