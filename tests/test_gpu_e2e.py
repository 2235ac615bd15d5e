"""End-to-end C1 (BASELINE configs[0], the reference's scripts/sanity_forward.py shapes: 4 x 1 s audio,
2-layer d_model 128 decoder with 4 heads, 32 tokens, T = 10) through the drop-in modules on the GPU:
AcousticEncoder -> jumpy sampler (T_infer 10, r 5, greedy MAP) -> token ids -> text (the reference
tokenizer's vocab) -> CER, against the same pipeline on the CPU oracle. The encoder output must match
the oracle's (1e-4); both samplers then start from the GPU encoder's output and the same x_T, so the
decoded ids — and therefore the CER — must be identical (north_star "CPU-parity CER on the
sanity_forward fixture"). The oracle's WavLM, decoder and sampler are pinned to the reference
(tests/test_oracle_golden.py); its decoder is head-count generic, the fixtures hold H = 2."""
import os

import pytest
import torch

from helpers import SMALL_WAVLM, _dec_sd, close
from oracle import fddm_oracle as O
from test_gpu_models import _encoder, make_decoder

pytestmark = pytest.mark.gpu
dev = torch.device("cuda:0")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("mode,graph", [("exact", False), ("exact", True), ("fast", False)])
def test_sanity_forward_cer_matches_cpu_oracle(mode, graph, monkeypatch):
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from fddm_hip import runtime as rt
    from models.evaluate import VocabTokenizer, _ids_to_text_one, calculate_cer
    from sampler import jumpy_sampler as JS

    V, d, H, NL, FF, B, L, Tn = 8000, 128, 4, 2, 2048, 4, 32, 10
    gen = torch.Generator().manual_seed(11)
    wave = 0.1 * torch.randn(B, 16000, generator=gen)
    x0 = torch.randint(4, V, (B, L), generator=gen)
    x0[1, 25:] = 0
    x0[3, 12:] = 0
    xT = torch.randint(0, V, (B, L), generator=gen)
    tok = VocabTokenizer(os.path.join(GOLDEN, "vocab_zhTW_A.json.gz"))

    with rt.use_precision("fp32"):
        enc = _encoder(SMALL_WAVLM, d)
        dec = make_decoder(V, d, H, NL, FF, dropout=0.1)
        dec.eval()
        cond, _, _ = enc(wave.to(dev))
        smp = JS.DiffusionJumpySampler(DiscreteDiffusionScheduler(K=V, T=Tn, device=dev, beta_max=0.2), dec, K=V,
                                       T_train=Tn, T_infer=Tn, r=5, greedy=True, posterior_mode="map",
                                       sampling_mode=mode, device=dev)
        monkeypatch.setattr(JS.torch, "randint", lambda low, high, size, device=None: xT.to(dev))
        x_pred, _ = smp.sample(cond, seq_len=L, graph=graph, return_probs=False)
    x_pred = x_pred.cpu()

    from helpers import wavlm_sd
    g = O.wavlm_geometry(**SMALL_WAVLM)
    cond_ref = O.acoustic_encoder(wavlm_sd(g, d), wave, g, d)
    assert cond.shape == (B, 49, d)
    close(cond, cond_ref, rtol=1e-4, what="C1 encoder output")

    sd = _dec_sd(V, d, H, NL, FF)
    c_cpu = cond.detach().cpu()
    b, ab = O.sched_tables(Tn, 0.2)

    def logits_fn(x, tv):
        with torch.no_grad():
            return O.decoder_forward(sd, x, tv, c_cpu, None, H=H, num_layers=NL)

    _, _, x_ref = O.jumpy_sample(logits_fn, xT, Tn, 5, b.numpy(), ab.numpy(), V, Tn, mode=mode)
    assert torch.equal(x_pred, x_ref), "decoded ids differ from the CPU oracle"

    def cer(pred):
        return sum(calculate_cer(_ids_to_text_one(x0[i], tok, 0), _ids_to_text_one(pred[i], tok, 0))
                   for i in range(B)) / B

    c_gpu, c_ref = cer(x_pred), cer(x_ref)
    assert c_gpu == c_ref
    assert c_gpu > 0.5  # random weights: the decode is noise, the test is about identical outputs


def test_real_data_loader_trains(tmp_path, monkeypatch):
    """The real-data path (data_io.CVZhTWDataset: WAV clips + SentencePiece ids rebuilt from the reference's .vocab)
    feeding train.train_one_epoch at C1 geometry: two steps from the DataLoader give the same KL values as the same two
    steps fed the expected (wav, ids) tensors directly (1e-5: the encoder's split-K and the LayerNorm parameter
    gradients accumulate with float atomics, so two identical runs agree to ~1e-7, not bit for bit), and the losses are
    finite."""
    import gzip
    import json

    import numpy as np

    import data_io
    import train as T_
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from fddm_hip import runtime as rt
    from fddm_hip.optim import FusedAdamW
    from models.projection import SpeechProjector, TextEmbedding, TextProjector
    from test_cpu_data import _write_wav
    from test_gpu_models import make_decoder

    monkeypatch.chdir(tmp_path)
    os.makedirs("clips")
    with gzip.open(os.path.join(GOLDEN, "spm_zhTW_A.vocab.gz")) as f:
        (tmp_path / "spm.vocab").write_bytes(f.read())
    rng = np.random.default_rng(5)
    texts = ["我們今天去高雄", "台北捷運交流道", "政府需要討論這個問題", "台中市的公車系統"]
    clips = []
    for i, s in enumerate(texts):
        x = rng.integers(-8000, 8000, size=(16000 * (1 + i % 2), 1))
        _write_wav(f"clips/{i}.wav", x, 16000)
        clips.append(x[:, 0])
    with open("m.json", "w", encoding="utf-8") as f:
        json.dump([{"processed_path": f"clips/{i}.wav", "normalized_sentence": s} for i, s in enumerate(texts)], f,
                  ensure_ascii=False)
    V, d, H, NL, FF, L, Tn = 8000, 128, 4, 2, 2048, 32, 10
    ds = data_io.CVZhTWDataset("m.json", "spm.model", max_len=L, pad_id=0)
    tok = data_io.load_tokenizer("spm.model")
    direct = []
    for b in range(2):
        w = torch.zeros(2, 320000)
        x0 = torch.zeros(2, L, dtype=torch.long)
        for j in range(2):
            i = 2 * b + j
            w[j, : clips[i].size] = torch.from_numpy((clips[i] / 32768.0).astype(np.float32))
            ids = tok.encode(texts[i])
            x0[j, : len(ids)] = torch.tensor(ids)
        direct.append((w, x0))

    def run(loader):
        kls = []
        with rt.use_precision("fp32"):
            torch.manual_seed(3)
            rt.reseed(3)
            from test_gpu_models import _encoder
            enc = _encoder(SMALL_WAVLM, d)
            dec = make_decoder(V, d, H, NL, FF, dropout=0.1)
            sp, te, tp = SpeechProjector(d, 256).to(dev), TextEmbedding(V, 256).to(dev), TextProjector(256, 256).to(dev)
            opt = FusedAdamW(list(dec.parameters()) + list(sp.parameters()) + list(te.parameters()) +
                             list(tp.parameters()), lr=2e-4, weight_decay=0.01)

            class Rec(T_.SchedulerAdapter):
                def kl_term(self, *a, **k):
                    v = super().kl_term(*a, **k)
                    kls.append(float(v.detach()))
                    return v

            cfg = T_.Config(seed=1, data={"pad_id": 0}, model={}, diffusion={"T": Tn}, inference={}, optim={},
                            lfd={"n_step_fd": 4, "tau": 1.0, "lambda_offdiag": 5e-3}, log={"log_every": 1000})
            sch = Rec(DiscreteDiffusionScheduler(K=V, T=Tn, device=dev))
            gs, loss = T_.train_one_epoch(enc, dec, sp, te, tp, sch, loader, opt, dev, cfg, 3, None, 1, False)
            torch.cuda.synchronize()
        assert gs == 5
        return kls

    got = run(torch.utils.data.DataLoader(ds, batch_size=2))
    want = run(direct)
    assert len(got) == 2 and all(np.isfinite(got))
    np.testing.assert_allclose(got, want, rtol=1e-5)
