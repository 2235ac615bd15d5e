"""DP gradient exchange overlapped with the decoder backward, on the GPU (fddm_hip.dist.OverlapReducer):
two ranks on cuda:0 (gloo moves the CUDA slices; RCCL on a multi-GPU node runs the same call sequence) each
run the decoder fwd + KL + backward on half of a batch with tiny buckets, so arena slices are all-reduced
while later blocks' backward kernels still accumulate. The averaged arena must equal the gradient of one
process on the whole batch (the KL loss is a batch mean; dropout 0; fp32 parity mode)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

V, d, H, NL, FF, S, L, T_STEPS = 1000, 128, 2, 3, 256, 24, 16, 10


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch():
    g = torch.Generator().manual_seed(11)
    B = 4
    x0 = torch.randint(1, V, (B, L), generator=g)
    x0[1, 12:] = 0
    x0[3, 9:] = 0
    xt = torch.randint(1, V, (B, L), generator=g)
    xt[x0 == 0] = 0
    t = torch.tensor([1, 4, 7, 10])
    cond = torch.randn(B, S, d, generator=g)
    return x0, xt, t, cond


def _grads(rank, world, bucket_bytes):
    import train as T_
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from fddm_hip import dist as fdist
    from fddm_hip import runtime as rt
    from fddm_hip.optim import FusedAdamW
    from test_gpu_models import make_decoder
    dev = torch.device("cuda:0")
    x0, xt, t, cond = _batch()
    sl = slice(None) if world == 1 else slice(2 * rank, 2 * rank + 2)
    x0, xt, t, cond = (v[sl].to(dev) for v in (x0, xt, t, cond))
    with rt.use_precision("fp32"):
        dec = make_decoder(V, d, H, NL, FF)
        dec.train()
        opt = FusedAdamW(list(dec.parameters()))
        opt.use_grad_arena(list(dec.parameters()), dec.grad_ready_order())
        red = fdist.OverlapReducer(opt.arena, bucket_bytes=bucket_bytes) if world > 1 else None
        sch = T_.SchedulerAdapter(DiscreteDiffusionScheduler(K=V, T=T_STEPS, device=dev))
        opt.zero_grad()
        logits = dec(xt, t, cond, x_mask=x0 != 0)
        loss = sch.kl_term(xt, x0, logits, t, x0 != 0)
        loss.backward()
        inflight = 0 if red is None else len(red.works)
        fdist.allreduce_grads(list(dec.parameters()))
        torch.cuda.synchronize()
    return {n: p.grad.detach().cpu().clone() for n, p in dec.named_parameters()}, inflight


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        gr, nin = _grads(rank, world, 64 << 10)
        q.put((rank, {n: v.numpy() for n, v in gr.items()}, nin))   # by value: the worker exits first
    finally:
        dist.destroy_process_group()


def test_overlapped_allreduce_matches_full_batch_gradient():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, gr, nin = q.get(timeout=100)
        got[r] = (gr, nin)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref, _ = _grads(0, 1, 0)
    assert got[0][1] > 1, "expected several slices in flight before backward finished"
    for n, g in ref.items():
        scale = g.abs().max().item() + 1e-12
        for r in range(world):
            err = (torch.from_numpy(got[r][0][n]) - g).abs().max().item() / scale
            assert err < 1e-4, f"{n} rank {r}: rel err {err:.2e}"


# ------------------------------------------------------------------ a full DP train step with a global-batch L_fd
SV, Sd, SH, SNL, SFF, SL, ST = 600, 128, 2, 2, 256, 20, 10
NOISE_ONLY = ("s_proj.proj.net.0.bias", "t_proj.proj.net.0.bias")


def _step_batches():
    g = torch.Generator().manual_seed(21)
    out = []
    for i in range(3):
        wave = 0.1 * torch.randn(4, 16000, generator=g)
        x0 = torch.randint(1, SV, (4, SL), generator=g)
        x0[1, 14:] = 0
        x0[2, 9:] = 0
        xt = torch.randint(1, SV, (4, SL), generator=g)
        t = (torch.tensor([1, 3, 7, 10]), torch.tensor([10, 2, 5, 1]), torch.tensor([4, 9, 2, 6]))[i]
        out.append((wave, x0, xt, t))
    return out


def _train_two_steps(rank, world, sync):
    """train_one_epoch over global steps 3 (KL), 4 (L_fd) and 5 (KL) on this rank's rows (all 4 when world == 1),
    encoder on its side stream, decoder gradients all-reduced by the overlapped reducer; returns final params, L_fd
    and the torch.distributed collectives the three steps issued (helpers.CollectiveLog)."""
    import train as T_
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from fddm_hip import runtime as rt
    from fddm_hip.optim import FusedAdamW
    from helpers import SMALL_WAVLM, CollectiveLog, _step_params
    from models.projection import SpeechProjector, TextEmbedding, TextProjector
    from test_gpu_models import _encoder, make_decoder
    dev = torch.device("cuda:0")
    sl = slice(None) if world == 1 else slice(2 * rank, 2 * rank + 2)
    data = [tuple(v[sl] for v in b) for b in _step_batches()]
    rec = []
    with rt.use_precision("fp32"):
        enc = _encoder(SMALL_WAVLM, Sd)
        dec = make_decoder(SV, Sd, SH, SNL, SFF)
        params = _step_params(SV, Sd, SNL, SFF, SH)
        sp, te, tp = SpeechProjector(Sd, 256), TextEmbedding(SV, 256), TextProjector(256, 256)
        for pre, m in (("s_proj.", sp), ("t_embed.", te), ("t_proj.", tp)):
            m.load_state_dict({n: params[pre + n] for n, _ in m.named_parameters()})
            m.to(dev)
        xq = iter([b[2].to(dev) for b in data])
        tq = iter([b[3].to(dev) for b in data])

        class TF(T_.SchedulerAdapter):
            def sample_q(self, x0, t):
                return next(xq)

        orig = T_.lfd_loss

        def rl(*a, **k):
            v = orig(*a, **k)
            rec.append(float(v.detach() if torch.is_tensor(v) else v))
            return v

        T_.lfd_loss = rl
        try:
            trainable = list(dec.parameters()) + list(sp.parameters()) + list(te.parameters()) + \
                list(tp.parameters())
            opt = FusedAdamW(trainable, lr=2e-4, weight_decay=0.01)
            cfg = T_.Config(seed=1, data={"pad_id": 0}, model={}, diffusion={"T": ST}, inference={}, optim={},
                            lfd={"n_step_fd": 4, "tau": 1.0, "lambda_offdiag": 5e-3, "sync_batch_stats": sync},
                            log={"log_every": 1000})
            sch = TF(DiscreteDiffusionScheduler(K=SV, T=ST, device=dev))
            with CollectiveLog() as cl:
                T_.train_one_epoch(enc, dec, sp, te, tp, sch, [(b[0], b[1]) for b in data], opt, dev, cfg, 3, None,
                                   1, False, draw_t=lambda B: next(tq))
                torch.cuda.synchronize()
        finally:
            T_.lfd_loss = orig
    final = {("decoder." + n): p.detach().cpu().clone() for n, p in dec.named_parameters()}
    for pre, m in (("s_proj.", sp), ("t_embed.", te), ("t_proj.", tp)):
        final.update({pre + n: p.detach().cpu().clone() for n, p in m.named_parameters()})
    return final, rec, params, cl.log


def _step_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import datetime
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    try:
        final, rec, _, log = _train_two_steps(rank, world, True)
        q.put((rank, {n: v.numpy() for n, v in final.items()}, rec, log))
    finally:
        dist.destroy_process_group()


def test_dp_train_step_global_batch_lfd_matches_full_batch():
    """Two ranks x 2 utterances through train_one_epoch (KL step, L_fd step, KL step; the projectors' grads are None
    on the KL steps on both ranks), encoder side stream on, lfd.sync_batch_stats: the global-batch L_fd, w_t mean and
    the averaged gradients make every rank's parameters equal those of one process on all 4 utterances
    (reference losses/fddm_losses.py:18-58, train.py:390 over the whole batch), and both ranks issue the identical
    collective sequence (names, shapes, dtypes, ops), the L_fd step's statistics reductions included."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_step_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, logs = {}, {}
    for _ in range(world):
        r, fin, rec, log = q.get(timeout=240)
        got[r] = (fin, rec)
        logs[r] = log
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert logs[0] == logs[1], "ranks issued different collective sequences"
    names = [e[0] for e in logs[0]]
    assert names.count("all_reduce") >= 3, logs[0]
    ref, ref_rec, init, _ = _train_two_steps(0, 1, False)
    assert len(ref_rec) == 1
    for r in range(world):
        assert len(got[r][1]) == 1
        assert abs(got[r][1][0] - ref_rec[0]) <= 1e-4 * abs(ref_rec[0]), (r, got[r][1], ref_rec)
        for n, p in ref.items():
            if n in NOISE_ONLY:
                continue
            a = torch.from_numpy(got[r][0][n]).double()
            da = ((a - init[n].double()) ** 2).sum().item()
            db = ((p.double() - init[n].double()) ** 2).sum().item()
            assert abs(da - db) <= 5e-3 * db + 1e-12, f"rank {r} {n}: update {da:.4e} vs {db:.4e}"
            if "in_proj_bias" not in n:
                assert ((a - p.double()).abs() > 4e-6).float().mean().item() < 0.02, f"rank {r} {n}"


# ------------------------------------------------------- the N > 1 benchmark path and the C2 geometry under DP
@pytest.mark.parametrize("world", [2, 4])
def test_bench_ranks_run_real_c2_steps(world):
    """`bench.py --gpus N` at C2 (not a dry run): N ranks (gloo, all on this box's GPU; the 8-GPU node runs the
    same code over RCCL, one GPU per rank) run warm-up and timed train steps with the overlapped gradient
    all-reduce, the HIP-graph encoder on its side stream and the CU caps (no collective reserve by default); the
    line reports n_gpus N / dpN, per-rank ms/step and the caps in force, a finite loss, and every replica ends with
    bit-identical parameters (BASELINE configs[2])."""
    import json
    import math
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FDDM_DIST_BACKEND="gloo", FDDM_DIST_TIMEOUT_S="300")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(world), "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--checksum"], cwd=root, env=env, capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    print(json.dumps({k: out[k] for k in ("value", "ms_per_step", "n_gpus", "avg_loss", "param_checksums")}))
    assert out["n_gpus"] == world and out["config"]["parallelism"] == f"dp{world}"
    assert out["config"]["global_batch"] == 32 * world
    assert math.isfinite(out["avg_loss"]) and out["value"] > 0
    assert len(out["rank_ms_per_step"]["per_rank"]) == world and out["cu_caps"]["coll"] == 0
    assert out["cu_caps"]["enc"] == out["cu_caps"]["ncu"] * 3 // 4   # no reserve by default (train.cu_caps)
    cs = out["param_checksums"]
    assert len(cs) == world and all(c == cs[0] for c in cs), cs


def _c2_dp_grads(rank, world, params_out=None):
    """Two teacher-forced train_one_epoch steps (global steps 3: KL, 4: L_fd with global-batch statistics) at the C2
    decoder geometry (6 layers, d_model 512, 8 heads, ff 2048, L 256, V 8000) over WavLM-base on 10 s audio, encoder
    graph-replayed on its side stream with the CU caps, on this rank's rows (all 4 when world == 1); returns the
    gradients clip_grad_norm_ sees at each step (after the DP average)."""
    import train as T_
    from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
    from fddm_hip import runtime as rt
    from fddm_hip.optim import FusedAdamW
    from helpers import _step_params
    from models.projection import SpeechProjector, TextEmbedding, TextProjector
    from test_gpu_models import _encoder, make_decoder
    dev = torch.device("cuda:0")
    V_, d_, H_, NL_, FF_, L_, T_n = 8000, 512, 8, 6, 2048, 256, 200
    g = torch.Generator().manual_seed(33)
    data = []
    for i in range(2):
        wave = 0.1 * torch.randn(4, 160000, generator=g)
        x0 = torch.randint(1, V_, (4, L_), generator=g)
        x0[1, 200:] = 0
        x0[3, 150:] = 0
        xt = torch.randint(1, V_, (4, L_), generator=g)
        t = torch.tensor([1, 50, 120, 200]) if i == 0 else torch.tensor([7, 2, 199, 64])
        data.append((wave, x0, xt, t))
    sl = slice(None) if world == 1 else slice(2 * rank, 2 * rank + 2)
    data = [tuple(v[sl] for v in b) for b in data]
    with rt.use_precision("fp32"):
        enc = _encoder({}, d_)
        dec = make_decoder(V_, d_, H_, NL_, FF_)
        params = _step_params(V_, d_, NL_, FF_, H_)
        sp, te, tp = SpeechProjector(d_, 256), TextEmbedding(V_, 256), TextProjector(256, 256)
        for pre, m in (("s_proj.", sp), ("t_embed.", te), ("t_proj.", tp)):
            m.load_state_dict({n: params[pre + n] for n, _ in m.named_parameters()})
            m.to(dev)
        named = [("decoder." + n, p) for n, p in dec.named_parameters()]
        for pre, m in (("s_proj.", sp), ("t_embed.", te), ("t_proj.", tp)):
            named += [(pre + n, p) for n, p in m.named_parameters()]
        xq = iter([b[2].to(dev) for b in data])
        tq = iter([b[3].to(dev) for b in data])

        class TF(T_.SchedulerAdapter):
            def sample_q(self, x0, t):
                return next(xq)

        opt = FusedAdamW([p for _, p in named], lr=2e-4, weight_decay=0.01)
        grads = []
        inner = opt.clip_and_step

        def snap(*a, **k):      # the averaged gradients: the DP step leaves the SUM, AdamW applies grad_scale = 1/W
            gs_ = k.get("grad_scale", 1.0)
            grads.append({n: (None if p.grad is None else (p.grad.detach() * gs_).cpu()) for n, p in named})
            return inner(*a, **k)

        opt.clip_and_step = snap
        cfg = T_.Config(seed=1, data={"pad_id": 0}, model={}, diffusion={"T": T_n}, inference={}, optim={},
                        lfd={"n_step_fd": 4, "tau": 1.0, "lambda_offdiag": 5e-3, "sync_batch_stats": True},
                        log={"log_every": 1000})
        sch = TF(DiscreteDiffusionScheduler(K=V_, T=T_n, device=dev))
        from train import GraphedEncoder
        assert GraphedEncoder.supported(enc)
        T_.train_one_epoch(enc, dec, sp, te, tp, sch, [(b[0], b[1]) for b in data], opt, dev, cfg, 3, None, 1, False,
                           draw_t=lambda B: next(tq))
        torch.cuda.synchronize()
    if params_out is not None:
        params_out.update({n: p.detach().cpu().clone() for n, p in named})
    return grads


def _c2_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import datetime
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=300))
    try:
        grads = _c2_dp_grads(rank, world)
        q.put((rank, [{n: (None if v is None else v.numpy()) for n, v in gr.items()} for gr in grads]))
    finally:
        dist.destroy_process_group()


def test_dp_c2_geometry_matches_full_batch():
    """The overlapped all-reduce at the C2 decoder geometry, beside the graph-replayed, CU-capped encoder stream:
    two ranks x 2 utterances give, at both steps (KL, then L_fd with global-batch statistics), the gradients of one
    process on all 4 utterances (fp32 parity mode, norm-wise 1e-4; same None pattern)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, gr = q.get(timeout=400)
        got[r] = gr
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _c2_dp_grads(0, 1)
    for i in range(2):
        G = sum(float((v.double() ** 2).sum()) for v in ref[i].values() if v is not None) ** 0.5
        for r in range(world):
            assert {n for n, v in got[r][i].items() if v is None} == {n for n, v in ref[i].items() if v is None}
            worst = 0.0
            for n, v in ref[i].items():
                if v is None or n in NOISE_ONLY:
                    continue
                e = float((torch.from_numpy(got[r][i][n]).double() - v.double()).norm())
                worst = max(worst, e / max(float(v.double().norm()), 1e-3 * G))
            print(f"step {i} rank {r}: worst grad rel err {worst:.2e}")
            assert worst < 1e-4


# ------------------------------------------------- RCCL on hardware: a world-size-1 "nccl" group with the DP path forced
def _rccl_worker(backend, port, q):
    """One process: (backend None) the plain single-GPU step, or a world-size-1 process group of `backend` with the DP
    exchange forced on (fddm_hip.dist.force_dp): rank-0 broadcast, the overlapped all-reduce issued from the backward's
    grads_ready callbacks, the global-batch L_fd statistics, 1/W in AdamW. Returns the gradients at both steps, the
    final parameters and the collectives issued."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import datetime
    import torch.distributed as dist
    from fddm_hip import dist as fdist
    from helpers import CollectiveLog
    if backend is not None:
        kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=0, world_size=1, timeout=datetime.timedelta(seconds=120), **kw)
        fdist.force_dp(True)
    try:
        final = {}
        with CollectiveLog() as cl:
            grads = _c2_dp_grads(0, 1, params_out=final)
        q.put(([{n: (None if v is None else v.numpy()) for n, v in gr.items()} for gr in grads],
               {n: v.numpy() for n, v in final.items()}, cl.log))
    finally:
        if backend is not None:
            dist.destroy_process_group()


def _spawn_one(backend):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(backend, _free_port(), q))
    p.start()
    out = q.get(timeout=400)
    p.join(timeout=60)
    assert p.exitcode == 0
    return out


def test_rccl_world1_forced_dp_step_matches_single_gpu():
    """RCCL executes this code's DP path on hardware before any multi-GPU node does (verdict r5 item 5): a world-size-1
    `nccl` group (init with device_id, as bench.py does), the DP exchange forced on, one KL step and one L_fd step with
    sync_batch_stats at the C2 decoder geometry beside the graph-replayed encoder stream. The same run over a world-1
    gloo group is the reference for the collective path (the all-reduce of one rank is the identity, so both must
    give the single-GPU result). The fp32 kernels' atomics make runs differ by ~1.5e-6 (KL step) and ~1e-5 (L_fd step)
    norm-wise even between two plain runs (tools/probe/rccl_diag.py: gloo vs gloo-bulk 7.7e-6 on the L_fd step), so
    the bar is that spread: gradients within 5e-5 of the gloo run and of the plain single-GPU step (whose L_fd
    statistics take the local kernels). Parameters after two AdamW steps within 1e-3 norm-wise: the update g / sqrt(v)
    has magnitude ~lr whatever |g| is, so elements whose gradient is at the noise level take noise-driven steps (two
    plain runs already differ by 1.9e-4 .. 2.8e-4 on the worst parameter, measured on MI355X). The two projector biases whose true
    gradient is zero (the L_fd standardisation removes them; NOISE_ONLY) are left out, as in the other DP tests.
    Not a scaling number: SCALE runs on the driver's 8-GPU node."""
    ref_g, ref_p, ref_log = _spawn_one(None)
    glo_g, glo_p, glo_log = _spawn_one("gloo")
    rc_g, rc_p, rc_log = _spawn_one("nccl")
    assert ref_log == [] and rc_log == glo_log, (rc_log[:8], glo_log[:8])
    names = [e[0] for e in rc_log]
    # rank-0 broadcasts, one overlapped slice per 16 MB of the 155.8 MB arena on each step, the L_fd statistics
    assert names.count("broadcast") >= 1 and names.count("all_reduce") >= 2 * 9, names
    exact, w_gloo, w_ref = 0, 0.0, 0.0

    def rel(x, y):
        return float((x - y).norm()) / max(float(y.norm()), 1e-12)

    for i in range(2):
        for n, v in ref_g[i].items():
            assert (rc_g[i][n] is None) == (v is None) == (glo_g[i][n] is None), n
            if v is None or n in NOISE_ONLY:
                continue
            a, g, r = (torch.from_numpy(x).double() for x in (rc_g[i][n], glo_g[i][n], v))
            exact += int(torch.equal(a, g))
            w_gloo, w_ref = max(w_gloo, rel(a, g)), max(w_ref, rel(a, r))
    p_gloo, p_ref, p_worst = 0.0, 0.0, ""
    for n, v in ref_p.items():
        if n in NOISE_ONLY:
            continue
        a, g, r = (torch.from_numpy(x).double() for x in (rc_p[n], glo_p[n], v))
        if max(rel(a, g), rel(a, r)) > max(p_gloo, p_ref):
            p_worst = n
        p_gloo, p_ref = max(p_gloo, rel(a, g)), max(p_ref, rel(a, r))
    print(f"RCCL world-1: {exact} gradient tensors bit-identical to the gloo run; worst gradient rel diff vs gloo "
          f"{w_gloo:.2e}, vs the single-GPU step {w_ref:.2e}; worst parameter rel diff {p_gloo:.2e} / {p_ref:.2e} ({p_worst})")
    assert w_gloo < 5e-5 and w_ref < 5e-5 and p_gloo < 1e-3 and p_ref < 1e-3
