"""C5 (BASELINE.json configs[4]) at its stated geometry: the jumpy sampler over the C2 model — WavLM-base encoder on
10 s audio, 6-layer d_model 512 / 8 heads decoder, V = 8000, seq_len 256, T_train 200, T_infer 20, r 5, exact
posterior, greedy (reference sampler/jumpy_sampler.py:167-293, fddm/sched/diffusion_scheduler.py:106-208,
models/evaluate.py:453-477), built exactly as `bench.py --config c5` builds it, on B = 2 utterances.

Per jump, the oracle restates the decoder forward from the GPU's own input x_t and acoustic condition (so a
near-tie decided differently at one jump does not make every later jump diverge) and the reference's exact
posterior argmax (oracle.jump_argmax, pinned by tests/golden/jumpy.npz); the GPU's x_{t-Δ} must equal it wherever
the posterior's relative margin between the two candidate tokens exceeds the tolerance, likewise x̂0 wherever its
top-2 logit gap does. The final decode (argmax of the last x̂0) gives the CER against random target ids through the
reference tokenizer's vocabulary; GPU and oracle CER are equal when no near-tie differs. The HIP-graph replay of
the whole denoise loop (the C5 benchmark path) must equal the eager loop."""
import os
from types import SimpleNamespace

import pytest
import torch

from helpers import close
from oracle import fddm_oracle as O

pytestmark = pytest.mark.gpu
dev = torch.device("cuda:0")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("prec,enc_tol,mtol", [("fp32", 1e-4, 1e-4), ("bf16", 5e-2, 5e-2)])
def test_c5_sampler_matches_oracle(prec, enc_tol, mtol, monkeypatch):
    import bench
    from fddm_hip import runtime as rt
    from models.evaluate import VocabTokenizer, _ids_to_text_one, calculate_cer
    from sampler import jumpy_sampler as JS

    args = SimpleNamespace(config="c5", batch=2, seconds=10.0, seq_len=256, layers=6, d_model=512, heads=8,
                           precision=prec)
    B, L, V = args.batch, args.seq_len, 8000
    gen = torch.Generator().manual_seed(21)
    wave = 0.1 * torch.randn(B, 160000, generator=gen)
    xT = torch.randint(0, V, (B, L), generator=gen)
    target = torch.randint(4, V, (B, L), generator=gen)
    target[1, 180:] = 0
    with rt.use_precision(prec):
        torch.manual_seed(7)
        _, _, models, _ = bench.build(args, dev)
        smp = bench.c5_sampler(models, dev)
        enc, dec = models[0], models[1]
        with torch.no_grad():
            cond = enc(wave.to(dev))[0]
        xs, x0hs = [xT.to(dev)], []
        plan = smp._plan(B)
        with torch.no_grad():
            for t, delta, coef in plan:
                nx, x0h, _ = smp._step(xs[-1], t, delta, cond, coef)
                xs.append(nx)
                x0hs.append(x0h)
        monkeypatch.setattr(JS.torch, "randint", lambda low, high, size, device=None: xT.to(dev))
        x0_graph, _ = smp.sample(cond, seq_len=L, graph=True, return_probs=False)
        torch.cuda.synchronize()
        enc_sd = {k: v.detach().float().cpu() for k, v in enc.state_dict().items()}
        sd = {k: v.detach().float().cpu() for k, v in dec.state_dict().items()}
        del models, smp, enc, dec
    assert [(t, d) for t, d, _ in plan] == [(20, 5), (15, 5), (10, 5), (5, 5)]
    assert torch.equal(x0_graph.cpu(), x0hs[-1].cpu()), "graph replay of the denoise loop differs from the eager loop"

    cref = O.acoustic_encoder(enc_sd, wave, O.wavlm_geometry(), args.d_model)
    close(cond.float(), cref, rtol=enc_tol, what=f"C5 {prec} encoder output")

    c_cpu = cond.detach().float().cpu()
    betas, _ = O.sched_tables(200)
    near = bad = 0
    last_ref = None
    for j, (t, delta, _) in enumerate(plan):
        x_in = xs[j].cpu()
        tv = torch.full((B,), t, dtype=torch.long)
        with torch.no_grad():
            logits = O.decoder_forward(sd, x_in, tv, c_cpu, None, H=args.heads, num_layers=args.layers)
        nx_ref, margin = O.jump_argmax(logits, x_in, tv, delta, betas.numpy(), V, 200)
        ok = margin.abs() >= mtol
        near += int((~ok).sum())
        bad += int((xs[j + 1].cpu() != nx_ref)[ok].sum())
        top2 = logits.double().topk(2, -1).values
        gap_ok = (top2[..., 0] - top2[..., 1]) >= mtol * top2[..., 0].abs().clamp_min(1.0)
        bad += int((x0hs[j].cpu() != logits.argmax(-1))[gap_ok].sum())
        last_ref = (logits.argmax(-1), gap_ok)
    print(f"C5 {prec}: {near} of {len(plan) * B * L} jump decisions within the margin tolerance {mtol:g}, "
          f"{bad} differing decisions beyond it")
    assert bad == 0
    tok = VocabTokenizer(os.path.join(GOLDEN, "vocab_zhTW_A.json.gz"))

    def cer(pred):
        return sum(calculate_cer(_ids_to_text_one(target[i], tok, 0), _ids_to_text_one(pred[i], tok, 0))
                   for i in range(B)) / B

    x_gpu, (x_ref, gap_ok) = x0hs[-1].cpu(), last_ref
    if torch.equal(x_gpu, x_ref):
        assert cer(x_gpu) == cer(x_ref)
    else:   # only near-ties differ (asserted above): each differing id moves the CER by at most one edit
        ndiff = int((x_gpu != x_ref).sum())
        assert abs(cer(x_gpu) - cer(x_ref)) <= ndiff / 100.0


def test_c5_full_batch_graph_replay_and_rows(monkeypatch):
    """C5 at its benchmark batch (B = 64, bf16): the HIP-graph replay of the whole denoise loop (the `bench.py
    --config c5` path) equals the eager loop on all 64 utterances, and two rows (first, last) of every jump agree
    with the oracle's decoder forward + exact posterior argmax on the GPU's own inputs beyond the bf16 margin."""
    import bench
    from fddm_hip import runtime as rt
    from sampler import jumpy_sampler as JS

    args = SimpleNamespace(config="c5", batch=64, seconds=10.0, seq_len=256, layers=6, d_model=512, heads=8,
                           precision="bf16")
    B, L, V, mtol = args.batch, args.seq_len, 8000, 5e-2
    gen = torch.Generator().manual_seed(23)
    wave = 0.1 * torch.randn(B, 160000, generator=gen)
    xT = torch.randint(0, V, (B, L), generator=gen)
    with rt.use_precision("bf16"):
        torch.manual_seed(7)
        _, _, models, _ = bench.build(args, dev)
        smp = bench.c5_sampler(models, dev)
        enc, dec = models[0], models[1]
        with torch.no_grad():
            cond = enc(wave.to(dev))[0]
        xs, x0hs = [xT.to(dev)], []
        plan = smp._plan(B)
        with torch.no_grad():
            for t, delta, coef in plan:
                nx, x0h, _ = smp._step(xs[-1], t, delta, cond, coef)
                xs.append(nx)
                x0hs.append(x0h)
        monkeypatch.setattr(JS.torch, "randint", lambda low, high, size, device=None: xT.to(dev))
        x0_graph, _ = smp.sample(cond, seq_len=L, graph=True, return_probs=False)
        torch.cuda.synchronize()
        sd = {k: v.detach().float().cpu() for k, v in dec.state_dict().items()}
        del models, smp, enc, dec
    assert torch.equal(x0_graph.cpu(), x0hs[-1].cpu()), "graph replay of the denoise loop differs from the eager loop"
    rows = [0, B - 1]
    c_cpu = cond.detach().float().cpu()[rows]
    betas, _ = O.sched_tables(200)
    bad = 0
    for j, (t, delta, _) in enumerate(plan):
        x_in = xs[j].cpu()[rows]
        tv = torch.full((len(rows),), t, dtype=torch.long)
        with torch.no_grad():
            logits = O.decoder_forward(sd, x_in, tv, c_cpu, None, H=args.heads, num_layers=args.layers)
        nx_ref, margin = O.jump_argmax(logits, x_in, tv, delta, betas.numpy(), V, 200)
        ok = margin.abs() >= mtol
        bad += int((xs[j + 1].cpu()[rows] != nx_ref)[ok].sum())
    assert bad == 0
