"""CPU tests of the host side: the C-ABI library loads and exports every declared symbol, the module
API keeps the reference's signatures and state_dict keys, and host-side integer logic (sampler
thresholds, rel-pos buckets, dropout streams) agrees with the oracle. No kernel is launched here."""
import inspect

import numpy as np
import torch

from helpers import SMALL_WAVLM, _dec_sd, wavlm_sd
from oracle import fddm_oracle as O


def test_library_exports_every_declared_symbol():
    from fddm_hip import _lib
    L = _lib.lib()
    names = _lib.declared_symbols()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), n
    assert L.fddm_abi_version() == 6
    assert b"no error" in L.fddm_error_string(0).lower()


def test_decoder_state_dict_keys_match_reference():
    from models.denoise_decoder import DenoisingTransformerDecoder
    dec = DenoisingTransformerDecoder(vocab_size=1000, d_model=128, nhead=2, num_layers=2, dim_ff=256, dropout=0.0)
    keys = set(dec.state_dict().keys())
    ref_keys = set(_dec_sd(1000, 128, 2, 2, 256).keys()) | {"pos_emb.inv_freq"}
    assert keys == ref_keys
    sig = inspect.signature(DenoisingTransformerDecoder.__init__)
    assert list(sig.parameters)[1:] == ["vocab_size", "d_model", "nhead", "num_layers", "dim_ff", "dropout", "max_len",
                                        "pad_id", "pos_emb_type", "use_film", "rope_base"]
    assert list(inspect.signature(DenoisingTransformerDecoder.forward).parameters)[1:] == \
        ["xt", "t", "cond", "x_mask", "c_mask"]


def test_encoder_state_dict_keys_match_hf_wavlm():
    from models.acoustic_encoder import AcousticEncoder
    enc = AcousticEncoder(wavlm_name=dict(SMALL_WAVLM), d_model=64)
    ours = set(enc.state_dict().keys())
    ref = set(wavlm_sd(O.wavlm_geometry(**SMALL_WAVLM), 64).keys())
    assert ref <= ours
    assert ours - ref == {"backbone.masked_spec_embed"}
    # same names as transformers' WavLMModel (third-party reference of the encoder arithmetic)
    from transformers import WavLMConfig, WavLMModel
    hf = WavLMModel(WavLMConfig(**SMALL_WAVLM))
    assert {"backbone." + k for k in hf.state_dict().keys()} == ours - {"proj.weight", "proj.bias"}


def test_scheduler_tables_and_thresholds_match_oracle():
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    s = DiscreteDiffusionScheduler(K=8000, T=200, device=torch.device("cpu"))
    b, ab = O.sched_tables(200)
    assert torch.equal(s.betas, b) and torch.equal(s.alpha_bar, ab)
    thr = s.sample_thresholds().numpy().view(np.uint32).astype(np.uint64)
    assert np.array_equal(thr, O.sample_thresholds(8000, ab))


def test_relbias_buckets_match_oracle():
    from fddm_hip import runtime as rt
    rel = torch.arange(-998, 999)
    assert torch.equal(rt.rel_bucket(rel, 320, 800), O.rel_position_bucket(rel, 320, 800))


def test_projection_and_loss_api():
    from losses.fddm_losses import lfd_loss
    from models.projection import SpeechProjector, TextEmbedding, TextProjector
    assert set(SpeechProjector(512, 256).state_dict()) == {"proj.net.0.weight", "proj.net.0.bias"}
    assert set(TextEmbedding(8000, 256).state_dict()) == {"proj.weight"}
    assert set(TextProjector(256, 256).state_dict()) == {"proj.net.0.weight", "proj.net.0.bias"}
    sig = inspect.signature(lfd_loss).parameters
    assert list(sig)[:4] == ["z_a", "z_b", "lambda_offdiag", "eps"]       # the reference's (fddm_losses.py:29)
    # additive: the data-parallel process group, keyword-only with a default (reference calls are unchanged)
    assert all(p.kind is p.KEYWORD_ONLY and p.default is None for p in list(sig.values())[4:])


def test_train_surface():
    import train
    assert [f for f in train.Config.__dataclass_fields__] == ["seed", "data", "model", "diffusion", "inference",
                                                               "optim", "lfd", "log"]
    params = list(inspect.signature(train.train_one_epoch).parameters)
    assert params[:13] == ["encoder", "decoder", "s_proj", "t_embed", "t_proj", "scheduler", "loader", "optimizer",
                           "device", "cfg", "global_step", "scaler", "epoch"]
    for m in ("sample_q", "kl_term", "w_t"):
        assert hasattr(train.SchedulerAdapter, m)


def test_align_speech_matches_oracle():
    import train
    z = torch.randn(2, 5, 3)
    for L in (3, 5, 8):
        assert torch.equal(train.align_speech(z, L), O.align_speech(z, L))


def test_dropout_stream_contract():
    # independent streams and the 16-bit threshold rate
    k1 = O.dropout_keep(1, 1, 200000, 0.1)
    k2 = O.dropout_keep(1, 2, 200000, 0.1)
    assert abs(k1.float().mean().item() - 0.9) < 0.005
    assert (k1 != k2).float().mean().item() > 0.1


def test_jumpy_sampler_api_and_plan():
    """DiffusionJumpySampler keeps the reference signature (jumpy_sampler.py:106-119, 238-243); the jump
    plan and the exact-mode coefficients (host fp32) equal the oracle's restatement bit for bit."""
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from sampler.jumpy_sampler import DiffusionJumpySampler
    sig = list(inspect.signature(DiffusionJumpySampler.__init__).parameters)[1:]
    assert sig == ["scheduler", "decoder", "K", "T_train", "T_infer", "r", "greedy", "posterior_mode", "sampling_mode",
                   "temperature", "device"]
    assert list(inspect.signature(DiffusionJumpySampler.sample).parameters)[1:4] == ["cond_c", "seq_len", "init"]
    cpu = torch.device("cpu")
    sch = DiscreteDiffusionScheduler(K=8000, T=200, device=cpu)
    b, _ = O.sched_tables(200)
    for T_inf, r in ((20, 5), (20, 3), (7, 7)):
        smp = DiffusionJumpySampler(sch, None, K=8000, T_train=200, T_infer=T_inf, r=r, device=cpu)
        plan = smp._plan(2)
        ts = [p[0] for p in plan]
        assert ts == list(range(T_inf, 0, -r)) and sum(p[1] for p in plan) == T_inf
        for t, d, coef in plan:
            ref = np.array(O.jump_coeffs(b.numpy(), 8000, 200, t, d), dtype=np.float32)
            assert np.array_equal(coef[0].numpy(), ref) and np.array_equal(coef[1].numpy(), ref)
    fast = DiffusionJumpySampler(sch, None, K=8000, T_train=200, T_infer=20, r=5, sampling_mode="fast", device=cpu)
    assert float(fast._plan(1)[0][2][0, 0]) == float(sch.alpha_bar[150])


def test_checkpoint_layout_and_resume_roundtrip(tmp_path):
    """save/load_checkpoint keep the reference's checkpoint keys (train.py:652-664) and restore weights,
    optimizer state and the dropout seed stream (torch.load weights_only)."""
    import train as T_
    from fddm_hip import runtime as rt
    from fddm_hip.optim import FusedAdamW
    from models.denoise_decoder import DenoisingTransformerDecoder
    from models.projection import SpeechProjector, TextEmbedding, TextProjector

    def build(seed):
        torch.manual_seed(seed)
        mods = (DenoisingTransformerDecoder(vocab_size=304, d_model=128, nhead=2, num_layers=1, dim_ff=256),
                SpeechProjector(128, 64), TextEmbedding(304, 64), TextProjector(64, 64))
        ps = [p for m in mods for p in m.parameters()]
        return mods, FusedAdamW(ps, lr=1e-3)

    (dec, sp, te, tp), opt = build(1)
    st = opt.state[next(iter(dec.parameters()))]
    st["step"], st["exp_avg"], st["exp_avg_sq"] = 3, torch.ones(1), torch.full((1,), 2.0)
    rt.reseed(77)
    rt.next_seed()
    path = str(tmp_path / "ep001.pt")
    T_.save_checkpoint(path, dec, sp, te, tp, step=42, epoch=1, raw={"seed": 1}, optimizer=opt)
    ck = torch.load(path, weights_only=True)
    assert {"decoder", "s_proj", "t_embed", "t_proj", "step", "epoch", "config"} <= set(ck)
    expect_next = rt.next_seed()
    (dec2, sp2, te2, tp2), opt2 = build(2)
    rt.reseed(5)
    step, epoch = T_.load_checkpoint(path, dec2, sp2, te2, tp2, opt2)
    assert (step, epoch) == (42, 1)
    for a, b in ((dec, dec2), (sp, sp2), (te, te2), (tp, tp2)):
        for (n, x), (_, y) in zip(a.state_dict().items(), b.state_dict().items()):
            assert torch.equal(x, y), n
    st2 = opt2.state[next(iter(dec2.parameters()))]
    assert st2["step"] == 3 and float(st2["exp_avg_sq"][0]) == 2.0
    assert rt.next_seed() == expect_next


def test_wavlm_checkpoint_loading_maps_legacy_names_strictly(tmp_path):
    """A local HF WavLM directory loads strictly: `wavlm.`-prefixed task checkpoints lose their heads, the
    legacy weight-norm names (weight_g / weight_v) of the positional conv map to the parametrization names, and
    a checkpoint of another geometry raises instead of leaving the frozen encoder partly random."""
    import json as _json

    import pytest
    from safetensors.torch import save_file
    from transformers import WavLMConfig, WavLMModel as HFWavLM
    from models.wavlm import WavLMModel
    torch.manual_seed(3)
    hf = HFWavLM(WavLMConfig(**SMALL_WAVLM)).eval()
    sd = {}
    for k, v in hf.state_dict().items():
        k = k.replace("parametrizations.weight.original0", "weight_g").replace("parametrizations.weight.original1",
                                                                              "weight_v")
        sd["wavlm." + k] = v.contiguous()
    sd["lm_head.weight"] = torch.zeros(3, 3)
    d = tmp_path / "wavlm"
    d.mkdir()
    save_file(sd, str(d / "model.safetensors"))
    (d / "config.json").write_text(_json.dumps(dict(SMALL_WAVLM, conv_dim=list(SMALL_WAVLM["conv_dim"]))))
    m = WavLMModel.from_pretrained(str(d))
    assert not m.random_init
    ours = m.state_dict()
    for k, v in hf.state_dict().items():
        assert torch.equal(ours[k], v), k
    bad = tmp_path / "bad"
    bad.mkdir()
    save_file({k: v for k, v in sd.items() if "pos_conv" not in k}, str(bad / "model.safetensors"))
    (bad / "config.json").write_text((d / "config.json").read_text())
    with pytest.raises(RuntimeError, match="does not match"):
        WavLMModel.from_pretrained(str(bad))
    assert WavLMModel.from_pretrained("microsoft/wavlm-large").random_init


def test_attention_dropout_contract_v2():
    """Attention-probability dropout draws (oracle attn_dropout_keep, csrc/attention.hip): keep rate 1 - p, rows
    and heads with different masks, no row a shifted copy of another, seeds and streams independent."""
    B, H, Lq, Lk, p = 2, 3, 64, 300, 0.1
    k = O.attn_dropout_keep(11, 1, B, H, Lq, Lk, p)
    assert k.shape == (B, H, Lq, Lk) and k.dtype == torch.bool
    assert abs(k.float().mean().item() - 0.9) < 0.01
    flat = k.reshape(-1, Lk).numpy()
    for r in range(0, flat.shape[0], 7):            # no row equals a shift of another (within the overlap)
        for s in range(r + 1, min(flat.shape[0], r + 40)):
            for d in (0, 4, 8):
                a, b = flat[r, d:], flat[s, :Lk - d]
                assert (a != b).mean() > 0.05
    k2 = O.attn_dropout_keep(11, 3, B, H, Lq, Lk, p)
    k3 = O.attn_dropout_keep(12, 1, B, H, Lq, Lk, p)
    assert (k != k2).float().mean().item() > 0.1 and (k != k3).float().mean().item() > 0.1
    # pairwise independence of neighbouring keys: P(both kept) ~ 0.81
    both = (k[..., 1:] & k[..., :-1]).float().mean().item()
    assert abs(both - 0.81) < 0.015


def test_attention_workspace_size_query():
    """fddm_attn_bwd_ws_floats (ABI 6): 64 floats per (b, h, query row) with Lq rounded up to 64 — the fused
    backward's f32 dQ partials for two key passes (csrc/attn7.hip bwdf7), the largest need of any backward kernel."""
    import ctypes
    from fddm_hip import _lib
    f = _lib.lib().fddm_attn_bwd_ws_floats
    f.restype = ctypes.c_long
    for B, H, Lq, Lk in ((32, 8, 256, 256), (32, 8, 256, 499), (16, 12, 512, 512), (1, 1, 1, 1), (2, 3, 65, 300)):
        assert f(B, H, Lq, Lk) == 64 * B * H * ((Lq + 63) // 64 * 64)


def test_wavlm_folded_gate_weights_match_summed_preactivations():
    """models/wavlm.py _fold_gate: the in-kernel WavLM gate (fddm_attn_fwd_relgate_x) uses the sums of
    gru_rel_pos_linear's rows 0-3 / 4-7 and of their biases; by linearity that equals summing the 8 pre-activations
    as HF modeling_wavlm.py:181-183 does (float64 check on random inputs)."""
    from models.wavlm import _fold_gate
    g = torch.Generator().manual_seed(5)
    lin = torch.nn.Linear(64, 8).double()
    with torch.no_grad():
        lin.weight.copy_(torch.randn(8, 64, generator=g, dtype=torch.float64))
        lin.bias.copy_(torch.randn(8, generator=g, dtype=torch.float64))
    x = torch.randn(100, 64, generator=g, dtype=torch.float64)
    pre = lin(x).detach()
    gw = _fold_gate(lin).double()
    assert gw.shape == (130,)
    ra = x @ gw[:64] + gw[128]
    rb = x @ gw[64:128] + gw[129]
    assert torch.allclose(ra, pre[:, :4].sum(-1), rtol=1e-6, atol=1e-5)
    assert torch.allclose(rb, pre[:, 4:].sum(-1), rtol=1e-6, atol=1e-5)
