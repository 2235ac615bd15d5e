"""GPU parity of the jumpy sampler: the fused `fddm_jump` step against the
reference's multi-step posterior argmax (golden fixture), full greedy sampler runs (exact and fast,
eager and HIP-graph replay) against the reference run, and the tempered Categorical draw against the
posterior distribution."""
import numpy as np
import pytest
import torch

from helpers import T, jumpy_case_inputs, load
from oracle import fddm_oracle as O

pytestmark = pytest.mark.gpu
dev = torch.device("cuda:0")
CASES = [([20, 20, 20, 20], 5), ([5, 5, 5, 5], 5), ([1, 1, 1, 1], 1), ([200, 150, 90, 7], 5), ([10, 12, 3, 40], 2),
         ([2, 30, 100, 199], 1)]


def _sched(K, Tn, device):
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    return DiscreteDiffusionScheduler(K=K, T=Tn, device=device, beta_max=0.2)


def test_jump_kernel_matches_reference_posterior_argmax():
    from fddm_hip import ops
    g = load("jumpy")
    sch = _sched(2000, 200, torch.device("cpu"))
    b, _ = O.sched_tables(200, 0.2)
    near = 0
    for i, (ts, delta) in enumerate(CASES):
        logits, xt = jumpy_case_inputs(i, 4, 48, 2000)
        t = torch.tensor(ts)
        d = min(delta, int(t.min()))
        coef = torch.stack(sch.multi_step_coeffs(t, d), 1).float().to(dev)
        nx, x0h = ops.jump(logits.reshape(-1, 2000).to(dev), xt.reshape(-1).to(dev), coef, 48)
        ref = T(g[f"c{i}_next"]).reshape(-1)
        _, margin = O.jump_argmax(logits, xt, t, delta, b.numpy(), 2000, 200)
        ok = margin.reshape(-1).abs() >= 1e-5
        near += int((~ok).sum())
        assert torch.equal(nx.cpu()[ok], ref[ok]), f"case {i}"
        assert torch.equal(x0h.cpu(), logits.reshape(-1, 2000).argmax(-1)), f"case {i} x0hat"
    assert near <= 3


@pytest.mark.parametrize("mode", ["exact", "fast"])
@pytest.mark.parametrize("graph", [False, True])
def test_jumpy_sampler_matches_reference_run(mode, graph, monkeypatch):
    """Greedy T_infer=20, r=5 run with the fixture's x_T: every jump's x_{t-Δ} and the final decode
    equal the reference's (decoder in the fp32 parity mode)."""
    from fddm_hip import runtime as rt
    from sampler import jumpy_sampler as JS
    from test_gpu_models import make_decoder
    g = load("jumpy")
    with rt.use_precision("fp32"):
        dec = make_decoder(1000, 128, 2, 2, 256, dropout=0.1)
        dec.eval()
        smp = JS.DiffusionJumpySampler(_sched(1000, 200, dev), dec, K=1000, T_train=200, T_infer=20, r=5,
                                       greedy=True, posterior_mode="map", sampling_mode=mode, device=dev)
        cond = T(g["run_cond"]).to(dev)
        xT = T(g[f"run_{mode}_xT"]).to(dev)
        # per-jump trajectory (eager)
        x = xT
        for j, (t, delta, coef) in enumerate(smp._plan(3)):
            assert (t, delta) == (int(g[f"run_{mode}_ts"][j]), int(g[f"run_{mode}_deltas"][j]))
            x, x0h, _ = smp._step(x, t, delta, cond, coef)
            assert torch.equal(x0h.cpu(), T(g[f"run_{mode}_x0hat"][j])), f"jump {j} x0hat"
            assert torch.equal(x.cpu(), T(g[f"run_{mode}_xs"][j])), f"jump {j}"
        # public entry point, x_T injected in place of torch.randint
        monkeypatch.setattr(JS.torch, "randint", lambda low, high, size, device=None: xT.clone())
        for _ in range(2 if graph else 1):
            x0, p = smp.sample(cond, seq_len=16, graph=graph)
            assert torch.equal(x0.cpu(), T(g[f"run_{mode}_x0"]))
        np.testing.assert_allclose(p.max(-1).values.cpu().numpy(), g[f"run_{mode}_plast_max"], rtol=1e-4)


@pytest.mark.parametrize("mode,temp", [("exact", 1.0), ("exact", 0.7), ("fast", 1.0)])
def test_jump_categorical_draw_matches_posterior(mode, temp):
    """greedy=False: draws over many identical rows follow the tempered posterior the reference's
    Categorical samples (jumpy_sampler.py:153-162): per-class frequencies within 5 sigma."""
    from fddm_hip import ops
    V, N, L = 16, 200000, 1000
    gen = torch.Generator().manual_seed(11)
    row = torch.randn(V, generator=gen) * 1.5
    xt_val = 3
    sch = _sched(V, 200, torch.device("cpu"))
    t, delta = torch.tensor([40]), 5
    p = torch.softmax(row, -1)
    if mode == "exact":
        oh = torch.zeros(1, 1, V)
        oh[0, 0, xt_val] = 1.0
        post = sch.q_posterior_multi_step(oh, p.view(1, 1, V), t, delta).view(V)
        coef = torch.stack(sch.multi_step_coeffs(t, delta), 1).float()
        m = ops.JUMP_SAMPLE
    else:
        ab = float(sch.alpha_bar[150])     # t_target 15 of T_infer 20 -> training step 150
        post = ab * p + (1 - ab) / V
        coef = torch.tensor([[ab, 0.0, 0.0, 0.0]])
        m = ops.JUMP_SAMPLE | ops.JUMP_FAST
    if temp != 1.0:
        post = torch.softmax(post.clamp_min(1e-12).log() / temp, -1)
    logits = row.expand(N, V).contiguous().to(dev)
    xt = torch.full((N,), xt_val, dtype=torch.long, device=dev)
    coef = coef.expand(N // L, 4).contiguous().to(dev)
    nx, _ = ops.jump(logits, xt, coef, L, mode=m, temperature=temp, seed=1234, rng_stream=7)
    freq = torch.bincount(nx.cpu(), minlength=V).double() / N
    sigma = (post.double() * (1 - post.double()) / N).sqrt()
    assert torch.all((freq - post.double()).abs() <= 5 * sigma + 1e-6), (freq, post)
