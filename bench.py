"""Benchmark: FDDM-ASR train-step utterances/sec on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "fddm_zhTW_base.yaml single MI355X"): WavLM-base encoder (random
init; pretrained weights are not available offline) + 6-layer d_model=512 / 8-head / ff 2048 decoder,
vocab 8000, T=200, dropout 0.1, n_step_fd=4, batch 32 x 10 s synthetic 16 kHz audio per GPU,
seq_len 256 random token targets (per-utterance length U{128..256}, pad tail). One step = the full
reference train step (train.py:340-443): encoder forward, q_sample, decoder fwd/bwd, KL, L_fd every 4th
step, clip + AdamW. Inputs are resident in HBM before the timed region. The frozen encoder of batch i+1
runs on a second HIP stream beside step i's decoder (train._encoded); every timed batch is encoded exactly
once inside the timed region (the first one without overlap).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4|c5]
  N>1: one rank per GPU over RCCL, per-GPU batch fixed ("weak"). Under torch.distributed.run (WORLD_SIZE set)
  the ranks come from the launcher; `python bench.py --gpus N` alone starts that launcher itself (a child
  process, before this process touches the GPU) and exits with its status. The world size the process group
  reports must equal N.
  --config c4: BASELINE configs[3] per GPU (12-layer d768 H12 decoder, seq 512, 16 utterances per GPU).
  --config c5: BASELINE configs[4], jumpy-sampler inference (B=64 x 10 s, T_infer 20, r 5, exact, greedy, seq 256,
  HIP-graph replay of the encoder and of the whole denoise loop): one "step" = encode + sample one batch; the line
  reports utterances/s and the RTF (replicas only across GPUs: inference exchanges nothing).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BF16_PEAK_TFLOPS = 2500.0       # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
F32_PEAK_TFLOPS = 157.3
HBM_PEAK_TBS = 8.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--config", choices=sorted(PRESETS), default="c2",
                    help="BASELINE.json workload: c2 = configs[1] (default), c4 = configs[3] per GPU, c5 = configs[4]")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--d-model", type=int, default=None)
    ap.add_argument("--heads", type=int, default=None)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=4)
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--lfd-sync", action="store_true",
                    help="DP: L_fd / w_t statistics over the global batch (lfd.sync_batch_stats)")
    ap.add_argument("--checksum", action="store_true",
                    help="report every rank's parameter checksum after the run (DP replicas must agree bit for bit)")
    ap.add_argument("--dry-run", action="store_true",
                    help="initialise the process group, report the launch shape, do no GPU work")
    return apply_preset(ap.parse_args())


# BASELINE.json workloads: (batch per GPU, seq_len, decoder layers, d_model, heads); explicit flags override
PRESETS = {"c2": (32, 256, 6, 512, 8), "c4": (16, 512, 12, 768, 12), "c5": (64, 256, 6, 512, 8)}


def apply_preset(args):
    for k, v in zip(("batch", "seq_len", "layers", "d_model", "heads"), PRESETS[args.config]):
        if getattr(args, k) is None:
            setattr(args, k, v)
    return args


def _free_port() -> int:
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def visible_gpus() -> int:
    """GPUs this process could use, counted without initialising HIP (the parent of `--gpus N` only launches the
    ranks): the KFD topology's GPU nodes (simd_count > 0), restricted by HIP/ROCR/CUDA_VISIBLE_DEVICES."""
    import glob
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            props = dict(line.split() for line in open(f) if len(line.split()) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(n: int) -> int:
    """`--gpus N` without a launcher: run this script under torch.distributed.run with N local ranks (one per
    GPU) as a child process and return its exit status. Nothing here initialises the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    import subprocess
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def gflop_per_utt(args, S=None):
    """Algorithmic GFLOP per utterance of one train step (necessary work, SURVEY §8(d) accounting: 2MNK per GEMM
    / conv, 4 Lq Lk d per attention forward; decoder backward = 2x forward minus the never-applied gradient into
    the frozen encoder's output (cross K/V projection dX, FiLM pooled dX); L_fd (fwd + bwd) amortised over
    n_step_fd = 4; WavLM's gated-bias attention is not in the survey's count (its SDPA call escapes
    torch.utils.flop_counter), so it is left out here too). Reproduces the survey's C2 193.87 / C4 491.68."""
    d, NL, L, V, FF, P = args.d_model, args.layers, args.seq_len, 8000, 2048, 256
    S = encoder_frames(args.seconds) if S is None else S
    n = int(16000 * args.seconds)
    conv = 0.0
    cin = 1
    for k, st in zip((10, 3, 3, 3, 3, 2, 2), (5, 2, 2, 2, 2, 2, 2)):
        n = (n - k) // st + 1
        conv += 2.0 * n * 512 * k * cin
        cin = 512
    E, EF = 768, 3072
    enc = conv + 2.0 * S * 512 * E + 2.0 * S * E * 48 * 128 + 12 * (2.0 * S * E * 4 * E + 4.0 * S * E * EF +
                                                                       2.0 * S * 64 * 8 * 12)
    if d != E:
        enc += 2.0 * S * E * d
    fwd = decoder_fwd_gflop(args, S) * 1e9
    bwd = 2.0 * fwd - NL * (2.0 * S * d * 2 * d + 4.0 * d * d)
    lfd_f = 2.0 * L * V * P + 2.0 * L * P * P + 2.0 * S * d * P + 2.0 * L * P * P
    lfd_b = 2 * 2.0 * L * V * P + 2 * 2.0 * L * P * P + 2.0 * S * d * P + 2 * 2.0 * L * P * P
    if getattr(args, "config", "c2") == "c5":     # inference: encoder + one decoder forward per jump
        return (enc + n_jumps(args) * fwd) / 1e9
    return (enc + fwd + bwd + (lfd_f + lfd_b) / 4) / 1e9


def decoder_fwd_gflop(args, S):
    """Decoder forward GFLOP per utterance (SURVEY §8(d) accounting)."""
    d, NL, L, V, FF = args.d_model, args.layers, args.seq_len, 8000, 2048
    blk = (2.0 * L * d * 3 * d + 4.0 * L * L * d + 2.0 * L * d * d + 2.0 * L * d * d + 2.0 * S * d * 2 * d +
           4.0 * L * S * d + 2.0 * L * d * d + 4.0 * d * d + 4.0 * L * d * FF)
    return (NL * blk + 2.0 * L * d * V + 2.0 * (4 * d * d * 2 + d * d)) / 1e9


T_INFER, JUMP_R = 20, 5      # C5: inference.T_infer / r (BASELINE configs[4])


def n_jumps(args):
    return -(-T_INFER // JUMP_R)


def build(args, device):
    import train as T_
    from fddm_hip import runtime as rt
    from fddm_hip.optim import FusedAdamW
    cfg = T_.Config(seed=1337, data={"pad_id": 0, "vocab_size": 8000},
                    model={"d_model": args.d_model, "nhead": args.heads, "num_layers": args.layers, "dim_ff": 2048,
                           "dropout": 0.1, "encoder": {"wavlm_name": {}, "freeze": True, "proj": "linear",
                                                       "pooling": "none"}, "projector": {"d_proj": 256}},
                    diffusion={"T": 200, "beta_max": 0.2}, inference={}, optim={"lr": 2e-4, "weight_decay": 0.01},
                    lfd={"n_step_fd": 4, "tau": 1.0, "lambda_offdiag": 5e-3}, log={"log_every": 10 ** 9})
    rt.set_precision(args.precision)
    models = T_.build_models(cfg, device)
    enc, dec, sp, te, tp, sch = models
    params = list(dec.parameters()) + list(sp.parameters()) + list(te.parameters()) + list(tp.parameters())
    opt = FusedAdamW(params, lr=2e-4, weight_decay=0.01)
    return T_, cfg, models, opt


def synthetic_batches(args, device, n, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    out = []
    B, L, V = args.batch, args.seq_len, 8000
    ns = int(16000 * args.seconds)
    for _ in range(n):
        wave = 0.1 * torch.randn(B, ns, device=device, generator=g)
        x0 = torch.randint(1, V, (B, L), device=device, generator=g)
        lens = torch.randint(L // 2, L + 1, (B,), device=device, generator=g)
        x0 = torch.where(torch.arange(L, device=device)[None] < lens[:, None], x0, torch.zeros_like(x0))
        out.append((wave, x0))
    return out


CONV1_SOURCES = ("gemm256.hip", "gemm.hip", "gemm.h", "lds_dma.h", "common.h")


def conv1_src_sha() -> str:
    """Hash of the kernel sources the dominant launch (conv layer 1 on gemm256) is compiled from: a committed PMC
    traffic figure is only valid for the kernel build it was measured on."""
    import hashlib
    h = hashlib.sha256()
    for f in CONV1_SOURCES:
        with open(os.path.join(ROOT, "fddm-asr_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(args):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (profiles/rNN_pmc_conv1.json, written by tools/pmc_traffic.py for this workload) — only a file measured on the
    current kernel sources (`kernel_src_sha`); otherwise (None, the reason)."""
    import glob
    sha = conv1_src_sha()
    stale = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_conv1.json")), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("batch") != args.batch or not d.get("traffic_bytes"):
            continue
        if d.get("kernel_src_sha") != sha:
            stale = stale or f"stale: {os.path.basename(path)} was measured on other kernel sources"
            continue
        return float(d["traffic_bytes"]), os.path.basename(path)
    return None, stale


def dominant_flops(args):
    """Algorithmic FLOPs of one launch of the dominant kernel: WavLM conv layer 1 as an implicit GEMM
    (M = B*T1 output frames, N = 512 channels, K = 3 taps * 512), the largest MFMA launch of the step."""
    T0 = (int(16000 * args.seconds) - 10) // 5 + 1
    T1 = (T0 - 3) // 2 + 1
    return 2.0 * args.batch * T1 * 512 * 3 * 512


def config_tag(args):
    geom = (args.layers, args.d_model, args.heads, args.seq_len, args.seconds)
    if args.config == "c5":
        return "C5 (BASELINE configs[4])" if geom == (6, 512, 8, 256, 10.0) and args.batch == 64 else "custom C5"
    if geom == (6, 512, 8, 256, 10.0) and args.batch == 32:
        return "fddm_zhTW_base C2"
    if geom == (12, 768, 12, 512, 10.0) and args.batch == 16:
        return "C4 (BASELINE configs[3], per GPU)"
    return "custom"


def workload_name(args):
    tag = config_tag(args)
    return (f"{tag}: WavLM-base + {args.layers}L d{args.d_model} H{args.heads} ff2048 decoder, V=8000, T=200, "
            f"dropout 0.1, n_step_fd=4")


def encoder_frames(seconds):
    n = int(16000 * seconds)
    for k, st in zip((10, 3, 3, 3, 3, 2, 2), (5, 2, 2, 2, 2, 2, 2)):
        n = (n - k) // st + 1
    return n


ATTN_PROBES = ("decoder.self_attn_fwd", "decoder.cross_attn_fwd", "decoder.self_attn_bwd", "decoder.cross_attn_bwd")


def decoder_attention(args, probes, peak):
    """Decoder attention launches timed with HIP events on their stream: algorithmic FLOPs per launch (dense
    Lq x Lk scores, head_dim = d_model / heads; forward 4 Lq Lk dh, backward 10 Lq Lk dh per (b, h): QK^T
    recompute, dP, dQ, dK, dV) / average launch time, against the dense bf16 MFMA peak (BASELINE north_star:
    >= 30 % on the decoder attention)."""
    L, S = args.seq_len, encoder_frames(args.seconds)
    dh = args.d_model // args.heads
    out = {}
    for name in ATTN_PROBES:
        ev = probes.get(name) or []
        if not ev:
            continue
        ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
        lk = L if "self" in name else S
        bwd = name.endswith("bwd")
        fl = (10 if bwd else 4) * args.batch * args.heads * L * lk * dh
        tf = fl / (ms * 1e-3) / 1e12
        # algorithmic HBM bytes (bf16 tensors): fwd reads Q, K, V and writes O; bwd reads Q, K, V, O, dO and writes
        # dQ, dK, dV (the per-row LSE / delta and the dropout keep words are < 2 % and left out)
        q_b, kv_b = 2.0 * args.batch * L * args.d_model, 2.0 * args.batch * lk * args.d_model
        byts = (4 * q_b + 4 * kv_b) if bwd else (2 * q_b + 2 * kv_b)
        hbm_us = byts / (HBM_PEAK_TBS * 1e12) * 1e6
        mfma_us = fl / (peak * 1e12) * 1e6
        row = {"avg_us": round(1e3 * ms, 1), "gflop_per_launch": round(fl / 1e9, 3), "tflops": round(tf, 1),
               "frac": round(tf / peak, 4), "launches": len(ev), "hbm_mb_per_launch": round(byts / 1e6, 1),
               "hbm_floor_us": round(hbm_us, 2), "mfma_floor_us": round(mfma_us, 2),
               # the best MFMA fraction a launch could reach when it must also move its bytes at HBM peak
               "attainable_frac": round(mfma_us / max(hbm_us, mfma_us), 4)}
        rep = probes.get(name + "#replay") or []
        if rep:   # the same launches replayed back to back on the step's tensors: kernel time without launch gaps
            kms = sum(a.elapsed_time(b) / n for a, b, n in rep) / len(rep)
            ktf = fl / (kms * 1e-3) / 1e12
            row.update({"kernel_us": round(1e3 * kms, 1), "kernel_tflops": round(ktf, 1),
                        "kernel_frac": round(ktf / peak, 4)})
        out[name.split(".", 1)[1]] = row
    return out


def param_checksums(models, world):
    """(sum of the raw fp32 bit patterns, float64 sum) of every trainable parameter, gathered from all ranks."""
    enc, dec, sp, te, tp, sch = models
    bits, tot = 0, 0.0
    for m in (dec, sp, te, tp):
        for p in m.parameters():
            x = p.detach().float().contiguous()
            bits += int(x.view(torch.int32).to(torch.int64).sum())
            tot += float(x.double().sum())
    mine = [bits, tot]
    if world == 1:
        return [mine]
    out = [None] * world
    dist.all_gather_object(out, mine)
    return out


def cpu_baseline(args, models):
    """The CPU oracle (plain torch fp32 restatement of the reference step) timed on the host cores on a
    bounded sample: 2 utterances of the same geometry, `cpu_steps` steps (kind "port")."""
    from oracle import fddm_oracle as O
    ncores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(ncores)
    nthreads = torch.get_num_threads()
    enc, dec, sp, te, tp, sch = models
    enc_sd = {k: v.detach().float().cpu() for k, v in enc.state_dict().items()}
    w = enc.backbone.encoder.pos_conv_embed.conv.weight.detach().float().cpu()
    geom = O.wavlm_geometry()
    params = {("decoder." + k): v.detach().float().cpu().clone() for k, v in dec.named_parameters()}
    for pre, m in (("s_proj.", sp), ("t_embed.", te), ("t_proj.", tp)):
        params.update({pre + k: v.detach().float().cpu().clone() for k, v in m.named_parameters()})
    betas, ab = O.sched_tables(200)
    opt = O.OracleAdamW()
    cfg = dict(d_model=args.d_model, nhead=args.heads, num_layers=args.layers, pad_id=0, n_step_fd=4, tau=1.0,
               lambda_offdiag=5e-3)
    g = torch.Generator().manual_seed(0)
    Bc, L = args.cpu_batch, args.seq_len
    ns = int(16000 * args.seconds)
    del w
    t0 = time.perf_counter()
    for i in range(args.cpu_steps):
        wave = 0.1 * torch.randn(Bc, ns, generator=g)
        x0 = torch.randint(1, 8000, (Bc, L), generator=g)
        t = torch.randint(1, 201, (Bc,), generator=g)
        xt = O.sample_xt(x0, t, 8000, ab, seed=i)
        O.oracle_train_step(params, enc_sd, geom, wave, x0, t, xt, cfg, opt, i + 4, betas, ab)
    dt = time.perf_counter() - t0
    return {"value": round(Bc * args.cpu_steps / dt, 4), "unit": "utterances/s", "cores": nthreads, "kind": "port",
            "torch_threads": nthreads, "affinity_cpus": len(os.sched_getaffinity(0)),
            "sample": f"oracle train step (CPU fp32 restatement), {args.cpu_steps} steps x {Bc} utt x "
                      f"{args.seconds:g} s, same geometry as the GPU line, global steps 4..{3 + args.cpu_steps} "
                      f"(L_fd on 1 in 4); {dt:.1f} s wall"}


def c5_sampler(models, device):
    from sampler.jumpy_sampler import DiffusionJumpySampler
    enc, dec, sp, te, tp, sch = models
    enc.eval()
    dec.eval()
    return DiffusionJumpySampler(sch.sch, dec, K=8000, T_train=200, T_infer=T_INFER, r=JUMP_R, greedy=True,
                                 posterior_mode="map", sampling_mode="exact", device=device)


def c5_cpu_baseline(args, models, smp):
    """The CPU oracle's C5 pipeline (WavLM restatement + decoder forward per jump + the reference's exact posterior
    argmax, oracle.jump_argmax) timed on the host cores on a bounded sample: 2 utterances of the same geometry."""
    from oracle import fddm_oracle as O
    ncores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(ncores)
    enc, dec, *_ = models
    enc_sd = {k: v.detach().float().cpu() for k, v in enc.state_dict().items()}
    sd = {k: v.detach().float().cpu() for k, v in dec.state_dict().items()}
    geom = O.wavlm_geometry()
    betas, ab = O.sched_tables(200)
    Bc = 2
    g = torch.Generator().manual_seed(0)
    wave = 0.1 * torch.randn(Bc, int(16000 * args.seconds), generator=g)
    xT = torch.randint(0, 8000, (Bc, args.seq_len), generator=g)
    t0 = time.perf_counter()
    with torch.no_grad():
        c = O.acoustic_encoder(enc_sd, wave, geom, args.d_model)
        O.jumpy_sample(lambda x, tv: O.decoder_forward(sd, x, tv, c, None, H=args.heads, num_layers=args.layers),
                       xT, T_INFER, JUMP_R, betas.numpy(), ab.numpy(), 8000, 200, mode="exact")
    dt = time.perf_counter() - t0
    return {"value": round(Bc / dt, 4), "unit": "utterances/s", "rtf": round(dt / (Bc * args.seconds), 5),
            "cores": torch.get_num_threads(), "kind": "port", "affinity_cpus": len(os.sched_getaffinity(0)),
            "sample": f"oracle C5 pipeline (CPU fp32 restatement: encoder + {n_jumps(args)} decoder forwards + exact "
                      f"posterior argmax), {Bc} utt x {args.seconds:g} s; {dt:.1f} s wall"}


def run_c5(args, device, world, rank):
    """C5: jumpy-sampler inference throughput. Per step: the frozen encoder over one resident batch (HIP-graph replay,
    conv layer 1 eager between the two graphs as in training) and the whole T_infer / r denoise loop replayed from one
    HIP graph (decoder forward + the fused posterior-argmax jump kernel per jump)."""
    from fddm_hip import runtime as rt
    from fddm_hip.graphs import GraphedEncoder
    T_, cfg, models, _ = build(args, device)
    enc = models[0]
    smp = c5_sampler(models, device)
    bb = enc.backbone
    bb.conv_cus = bb.conv_cus_rest = 0       # nothing runs beside the encoder here: whole chip
    ge = GraphedEncoder(enc) if GraphedEncoder.supported(enc) else None
    waves = [w for w, _ in synthetic_batches(args, device, 2, 3000 + rank)]

    def step(i):
        with torch.no_grad():
            w = waves[i % 2]
            c = ge.run(w, i % 2) if ge is not None else enc(w)[0]
            x0, _ = smp.sample(c, seq_len=args.seq_len, graph=True, return_probs=False)
        return x0

    for i in range(max(1, args.warmup)):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record()
    with rt.probing(["wavlm.conv1"]) as probes:
        for i in range(args.steps):
            step(i)
    ev[1].record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        tt = torch.tensor([el], device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    utt = args.batch * args.steps * world
    value = utt / el
    if rank == 0:
        pev = probes["wavlm.conv1"]
        kms = sum(a.elapsed_time(b) for a, b in pev) / max(1, len(pev))
        kflops = dominant_flops(args)
        achieved = kflops / (kms * 1e-3) / 1e12
        peak = BF16_PEAK_TFLOPS if args.precision == "bf16" else F32_PEAK_TFLOPS
        gpu_utt = gflop_per_utt(args)
        cpu = None if (args.no_cpu_baseline or world > 1) else c5_cpu_baseline(args, models, smp)
        out = {
            "metric": "jumpy-sampler inference utterances/sec (C5: 10 s @16 kHz, T_infer 20, r 5, exact, greedy, "
                      "seq_len 256)",
            "value": round(value, 2), "unit": "utterances/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000.0 * el / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "rtf": round(el / args.steps / (args.batch * args.seconds), 8),
            "data": "synthetic (random-init WavLM-base + decoder, random audio)",
            "config": {"workload": workload_name(args) + f", jumpy sampler T_infer {T_INFER} r {JUMP_R} exact greedy, "
                                                         "HIP-graph encoder + denoise loop",
                       "global_batch": args.batch * world, "seq_len": args.seq_len, "audio_seconds": args.seconds,
                       "parallelism": f"replicas{world}"},
            "roofline": {"bound": "mfma", "kernel": "WavLM conv layer 1 implicit GEMM (gemm256_kernel: persistent "
                                                    "256x256, GELU)", "achieved": round(achieved, 1), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": None,
                         "avg_ms": round(kms, 4), "launches_timed": len(pev), "flops_per_launch": kflops},
            "step_mfma_frac": round(value / world * gpu_utt / 1e3 / peak, 4),
            "gflop_per_utt": round(gpu_utt, 2),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    # FDDM_DIST_BACKEND=gloo rehearses the N > 1 path with every rank on one GPU (local % device_count);
    # the driver's multi-GPU runs use the default: RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("FDDM_DIST_BACKEND", "nccl")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if backend == "nccl" and not args.dry_run and visible_gpus() < args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but only {visible_gpus()} GPU(s) visible")
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: launcher started {world} rank(s) but --gpus is {args.gpus}")
    if world > 1:
        from datetime import timedelta
        timeout = timedelta(seconds=int(os.environ.get("FDDM_DIST_TIMEOUT_S", "600")))
        if args.dry_run:
            dist.init_process_group("gloo", timeout=timeout)
        else:
            if backend != "nccl":
                local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
            else:
                dist.init_process_group(backend, timeout=timeout)
        world = dist.get_world_size()
        if world != args.gpus:
            sys.exit(f"bench.py: process group has {world} rank(s), --gpus is {args.gpus}")
    if args.dry_run:
        if rank == 0:
            print(json.dumps({"n_gpus": world, "parallelism": f"dp{world}", "backend": backend,
                              "global_batch": args.batch * world}), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    device = torch.device("cuda", local)
    torch.manual_seed(1337)         # one model init on every rank (train_one_epoch also broadcasts rank 0's weights)
    if args.config == "c5":
        return run_c5(args, device, world, rank)
    T_, cfg, models, opt = build(args, device)
    if args.lfd_sync:
        cfg.lfd["sync_batch_stats"] = True
    from fddm_hip import runtime as rt
    rt.reseed(1337 + rank)
    enc, dec, sp, te, tp, sch = models
    batches = synthetic_batches(args, device, 4, 1000 + rank)
    loader_w = [batches[i % 4] for i in range(args.warmup)]
    loader_t = [batches[i % 4] for i in range(args.steps)]
    # the first warmup step is an L_fd step (global step % n_step_fd == 0, reference train.py:372): its one-time costs
    # (first launches of the L_fd kernels, allocator growth) stay out of the timed region for every W >= 1
    gs = cfg.lfd["n_step_fd"]
    gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, loader_w, opt, device, cfg, gs, None, 0, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    T_.ALLREDUCE_TAIL = [] if world > 1 else None   # DP: end of backward -> all gradient slices reduced
    t0 = time.perf_counter()
    with rt.probing(["wavlm.conv1"]) as probes:   # HIP events around the dominant launch, on its stream
        gs, avg_loss = T_.train_one_epoch(enc, dec, sp, te, tp, sch, loader_t, opt, device, cfg, gs, None, 1, False)
    host_s = T_.LAST_ENQUEUE_DONE - t0     # host enqueue time of the K steps (before the epoch's closing loss read)
    torch.cuda.synchronize()
    tail_ev, T_.ALLREDUCE_TAIL = T_.ALLREDUCE_TAIL, None
    el = time.perf_counter() - t0
    rank_ms = [1000.0 * el / args.steps]
    if world > 1:
        dist.barrier()
        tt = torch.zeros(world, device=device)
        tt[rank] = el
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)      # every rank's own time (the line reports min / max)
        rank_ms = [1000.0 * float(x) / args.steps for x in tt.tolist()]
        el = max(float(x) for x in tt.tolist())
    # decoder attention launches: HIP events on one extra, untimed step (an event pair around every attention
    # launch inside the timed steps would add its own stream gaps to ms_per_step)
    # the same step with the encoder not overlapped (FDDM_NO_ENC_PIPELINE) also times the dominant launch alone
    # on the whole chip ("roofline_isolated"; inside the timed steps it shares the GPU with the decoder)
    os.environ["FDDM_NO_ENC_PIPELINE"] = "1"
    try:
        with rt.probing(["wavlm.conv1", *ATTN_PROBES], replays=5) as aprobes:
            T_.train_one_epoch(enc, dec, sp, te, tp, sch, loader_t[:1], opt, device, cfg, gs, None, 2, False)
        torch.cuda.synchronize()
    finally:
        del os.environ["FDDM_NO_ENC_PIPELINE"]
    utt = args.batch * args.steps * world
    value = utt / el
    ms_step = 1000.0 * el / args.steps
    checks = param_checksums(models, world) if args.checksum else None
    if rank == 0:
        ev = probes["wavlm.conv1"]
        kms = sum(a.elapsed_time(b) for a, b in ev) / max(1, len(ev))
        kflops = dominant_flops(args)
        ncu = torch.cuda.get_device_properties(device).multi_processor_count
        caps = T_.cu_caps(device)
        conv_cus = caps["conv"]
        traffic, traffic_src = pmc_traffic(args)
        peak = BF16_PEAK_TFLOPS if args.precision == "bf16" else F32_PEAK_TFLOPS
        achieved = kflops / (kms * 1e-3) / 1e12
        iev = aprobes["wavlm.conv1"]
        iso_ms = sum(a.elapsed_time(b) for a, b in iev) / max(1, len(iev))
        iso = kflops / (iso_ms * 1e-3) / 1e12
        gpu_utt = gflop_per_utt(args)
        step_tflops = value / world * gpu_utt / 1e3
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args, models)
        out = {
            "metric": "train-step utterances/sec (10 s @16 kHz, seq_len 256) at 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "utterances/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.precision, "data": "synthetic (random-init WavLM-base, random audio/tokens)",
            "config": {"workload": workload_name(args),
                       "global_batch": args.batch * world, "seq_len": args.seq_len, "audio_seconds": args.seconds,
                       "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "kernel": "WavLM conv layer 1 implicit GEMM (gemm256_kernel: persistent 256x256, GELU)",
                         "achieved": round(achieved, 1), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_unit": "B/launch",
                         "traffic_source": traffic_src, "avg_ms": round(kms, 4),
                         "launches_timed": len(ev), "flops_per_launch": kflops,
                         # inside the timed steps the conv feature extractor's persistent GEMMs are capped to this many
                         # CUs (the decoder forward runs on the rest, train._encoded); frac_of_cus = achieved against
                         # that share of the chip's peak
                         "cus": conv_cus, "frac_of_cus": round(achieved / (peak * conv_cus / ncu), 4)},
            "roofline_isolated": {"kernel": "same launch, encoder not overlapped with the decoder, whole chip (untimed step)",
                                  "achieved": round(iso, 1), "frac": round(iso / peak, 4), "avg_ms": round(iso_ms, 4)},
            "decoder_attention": decoder_attention(args, aprobes, peak),
            "step_mfma_frac": round(step_tflops / peak, 4),
            "step_tflops": round(step_tflops, 1),
            "host_ms_per_step": round(1000.0 * host_s / args.steps, 3),
            "gflop_per_utt": round(gpu_utt, 2),
            "lfd_batch_stats": "global" if (args.lfd_sync and world > 1) else "local",
            "avg_loss": round(avg_loss, 4),
            "cpu_baseline": cpu,
        }
        out["cu_caps"] = caps        # persistent encoder GEMM caps beside the decoder; coll = reserve under DP
        if world > 1:
            out["rank_ms_per_step"] = {"min": round(min(rank_ms), 3), "max": round(max(rank_ms), 3),
                                       "per_rank": [round(x, 3) for x in rank_ms]}
        if tail_ev:
            # the part of the gradient all-reduce that outlasts the backward (DESIGN §5's overlap), per step
            tl = [a.elapsed_time(b) for a, b in tail_ev]
            out["allreduce_tail_ms"] = {"avg": round(sum(tl) / len(tl), 3), "max": round(max(tl), 3),
                                        "steps": len(tl)}
        if checks is not None:
            out["param_checksums"] = checks
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
