"""FDDM-ASR training entry point on MI355X (drop-in for the reference's train.py).

Keeps the reference surface: `python train.py --config configs/fddm_zhTW_base.yaml [--device]`, the
`Config` dataclass (exactly the 8 top-level YAML keys), `SchedulerAdapter` (sample_q / kl_term / w_t)
and `train_one_epoch(...)` with the same arguments and return value, and the checkpoint layout
(`decoder`, `s_proj`, `t_embed`, `t_proj`, `epoch`, `step`, `config`).

The step itself (train.py:340-443 of the reference) runs on libfddm_hip: fused q_sample draw, fused
categorical KL, fused decoder blocks, fused L_fd, fused clip+AdamW; optional data-parallel gradient
all-reduce over RCCL (fddm_hip.dist) when torch.distributed is initialised.
"""
from __future__ import annotations

import argparse
import logging
import os
import random
import time
import weakref
from dataclasses import dataclass
from datetime import datetime

import torch
import yaml

from fddm.sched.diffusion_scheduler import DiscreteDiffusionScheduler
from fddm_hip import dist as fdist
from fddm_hip import functions as FN
from fddm_hip import runtime as rt
from fddm_hip._lib import lib as _fddm_lib
from fddm_hip.graphs import GraphedEncoder, StepGraphs
from fddm_hip.optim import FusedAdamW
from losses.fddm_losses import lfd_loss
from models.acoustic_encoder import AcousticEncoder
from models.denoise_decoder import DenoisingTransformerDecoder
from models.projection import SpeechProjector, TextEmbedding, TextProjector

try:
    from tqdm import tqdm
except Exception:  # pragma: no cover
    tqdm = None


@dataclass
class Config:
    """YAML schema of configs/fddm_zhTW_base.yaml (reference train.py:164-173)."""
    seed: int
    data: dict
    model: dict
    diffusion: dict
    inference: dict
    optim: dict
    lfd: dict
    log: dict


class SchedulerAdapter:
    """train.py:176-273 of the reference. Dispatches to the fused kernels when the scheduler offers
    them (same hasattr style as the reference's w_t)."""

    def __init__(self, scheduler):
        self.sch = scheduler

    def sample_q(self, x0: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        if hasattr(self.sch, "sample_xt"):
            return self.sch.sample_xt(x0, t, rt.next_seed())
        B, L = x0.shape
        onehot = torch.zeros(B, L, self.sch.K, device=x0.device)
        onehot.scatter_(-1, x0.unsqueeze(-1), 1.0)
        p = self.sch.q_sample(onehot, t)
        return torch.multinomial(p.view(-1, self.sch.K), 1).view(B, L)

    def kl_term(self, xt, x0, logits_x0, t, x_mask=None) -> torch.Tensor:
        if not hasattr(self.sch, "betas"):
            raise ValueError("scheduler must provide betas [T] to build the posterior")
        mask = None
        if x_mask is not None:   # masked mean over L (train.py:247-251), reduced on the device with the KL
            mask = x_mask.contiguous().view(torch.uint8) if x_mask.dtype == torch.bool else \
                (x_mask != 0).contiguous().view(torch.uint8)
            mask = mask.reshape(-1)
        betas = self.sch.betas
        if betas.device != logits_x0.device or betas.dtype != torch.float32:
            betas = betas.to(logits_x0.device).float().contiguous()
        return FN.KLFn.apply(logits_x0.float(), xt, x0, t, mask, betas)

    def w_t(self, t: torch.Tensor) -> torch.Tensor:
        if hasattr(self.sch, "alpha_bar"):
            return self.sch.alpha_bar.to(t.device)[t - 1]
        if hasattr(self.sch, "w_prefix"):
            return self.sch.w_prefix.to(t.device)[t - 1]
        if hasattr(self.sch, "betas"):
            cp = torch.cumprod(1.0 - self.sch.betas.to(t.device), 0)
            return cp[t - 1]
        return torch.ones_like(t, dtype=torch.float32)


def align_speech(z_speech: torch.Tensor, L: int) -> torch.Tensor:
    """train.py:382-387: truncate, or repeat the last frame."""
    S = z_speech.size(1)
    if S >= L:
        return z_speech[:, :L, :]
    return torch.cat([z_speech, z_speech[:, -1:, :].repeat(1, L - S, 1)], dim=1)


def cu_caps(dev) -> dict:
    """CU caps of the encoder's persistent GEMMs while they run beside the decoder (_encoded): "enc" for the
    transformer layers (FDDM_ENC_CUS, default 3/4 of the chip), "conv" / "conv_rest" for conv layer 1 / layers 2-6
    (FDDM_ENC_CUS_CONV / _CONV2, default half). FDDM_COLL_CUS (default 0) lowers every cap by that many CUs, left
    free of persistent workgroups for RCCL's all-reduce kernels under data parallelism. It stays 0 by default: the
    caps sit on tile-round boundaries — the WavLM projections have 189 / 567 / 756 tiles of 256^2, 1 / 3 / 4 rounds
    at 192 CUs; at 184 the 189-tile launches take 2 rounds — and on one GPU the caps a reserve of 8 leaves (184 /
    120) made the C2 step 12 % slower (9.70 -> 10.88 ms, tools/probe/dpcaps.sh), against an unmeasured gain for the
    collectives, which run on their own stream beside the decoder's short launches."""
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    coll = int(os.environ.get("FDDM_COLL_CUS", 0))
    enc = int(os.environ.get("FDDM_ENC_CUS", ncu * 3 // 4))
    conv = int(os.environ.get("FDDM_ENC_CUS_CONV", ncu // 2))
    conv_rest = int(os.environ.get("FDDM_ENC_CUS_CONV2", conv))
    low = lambda c: max(8, c - coll)  # noqa: E731
    return {"enc": low(enc), "conv": low(conv), "conv_rest": low(conv_rest), "coll": coll, "ncu": ncu}


def _encoded(encoder, loader, device, optimizer):
    """Yields (c, c_mask, x0) per batch. The encoder is frozen (eval mode, none of its parameters in the
    optimizer; train.py:543), so its output for batch i+1 does not depend on step i: on a GPU it is computed
    on a second HIP stream, enqueued before step i's decoder work, and the two run concurrently (the persistent
    encoder GEMMs fill the CUs the decoder's small, latency-bound launches leave idle). Every batch is still
    encoded exactly once, in order; the consumer stream waits on the encoder's event before using c."""
    opt_ids = set(id(p) for g in optimizer.param_groups for p in g["params"])
    frozen = not any(id(p) in opt_ids for p in encoder.parameters())
    dev = torch.device(device)
    if dev.type != "cuda" or not frozen or os.environ.get("FDDM_NO_ENC_PIPELINE"):
        bb = getattr(encoder, "backbone", None)
        if bb is not None and getattr(bb, "conv_cus", 0):
            bb.conv_cus = bb.conv_cus_rest = 0  # nothing runs beside it: the conv GEMMs get the whole chip
        for wave, x0 in loader:
            wave = wave.to(device, non_blocking=True)
            x0 = x0.to(device, non_blocking=True)
            c, c_mask, _ = encoder(wave)
            yield c, c_mask, x0
        return
    main = torch.cuda.current_stream(dev)
    side = _enc_stream(dev)
    # persistent encoder GEMMs on 3/4 of the CUs (measured: 192 of 256 beats 256, 224, 208, 176 and 160), the conv
    # feature extractor's on half (it runs beside the decoder forward; bench.py C2 step, tools/cap_sweep.sh: conv
    # cap 128 -> 10.85-10.91 ms, 112 / 120 / 136 / 144 / 160 -> 11.0-11.06, 192 (= the rest) 11.02-11.11, 256
    # 11.17, 64 12.4)
    caps = cu_caps(dev)
    enc_cus, conv_cus = caps["enc"], caps["conv"]
    bb = getattr(encoder, "backbone", None)
    if bb is not None and hasattr(bb, "stage_rest"):
        bb.conv_cus = conv_cus
        bb.conv_cus_rest = caps["conv_rest"]   # conv layers 2..6
    # HIP-graph replay of the encoder forward (fddm_hip.graphs): the host launch path, not the GPU, bounded the step
    graphs = None
    if os.environ.get("FDDM_ENC_GRAPH", "1") != "0" and GraphedEncoder.supported(encoder):
        graphs = _ENC_GRAPHS.get(encoder)
        if graphs is None:
            graphs = _ENC_GRAPHS[encoder] = GraphedEncoder(encoder)
    nbatch = [0]

    def launch(batch):
        wave, x0 = batch
        wave = wave.to(device, non_blocking=True)
        x0 = x0.to(device, non_blocking=True)
        side.wait_stream(main)                  # inputs (and memory the main stream freed) are ready
        prev = _fddm_lib().fddm_gemm_persistent_cap(enc_cus)
        try:
            with torch.cuda.stream(side):
                if graphs is not None:
                    c, c_mask = graphs.run(wave, nbatch[0] % 2, enc_cus), None
                else:
                    c, c_mask, _ = encoder(wave)
            nbatch[0] += 1
        finally:
            _fddm_lib().fddm_gemm_persistent_cap(prev)
        with torch.cuda.stream(side):
            ev = torch.cuda.Event()
            ev.record(side)
        wave.record_stream(side)
        return c, c_mask, x0, ev

    it = iter(loader)
    nxt = next(it, None)
    pending = launch(nxt) if nxt is not None else None
    while pending is not None:
        c, c_mask, x0, ev = pending
        main.wait_event(ev)
        c.record_stream(main)
        if c_mask is not None:
            c_mask.record_stream(main)
        nxt = next(it, None)
        pending = launch(nxt) if nxt is not None else None
        yield c, c_mask, x0


LAST_ENQUEUE_DONE = 0.0
CLIP_MAX_NORM = 5.0     # clip_grad_norm_ max_norm of the reference step (train.py:411,422)
_STEP_GRAPHS = weakref.WeakKeyDictionary()    # decoder -> StepGraphs (HIP-graph replay of the decoder step)
# DP all-reduce tail (bench.py --gpus N): HIP events on the compute stream at the end of backward and after
# allreduce_grads (the stream has waited for every gradient slice); ALLREDUCE_TAIL collects the event pairs
ALLREDUCE_TAIL: list | None = None


def _mark_allreduce_tail(start=None):
    """Records the tail probe's events when bench.py enabled it (ALLREDUCE_TAIL is a list) and the run is DP."""
    if ALLREDUCE_TAIL is None or fdist.world() <= 1:
        return None
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    if start is not None:
        ALLREDUCE_TAIL.append((start, ev))
    return ev
_ENC_STREAMS: dict = {}
_ENC_GRAPHS = weakref.WeakKeyDictionary()     # encoder -> GraphedEncoder (released with the encoder)


def _step_graph_ok(device, scaler, optimizer, arena) -> bool:
    """HIP-graph replay of the decoder step (fddm_hip.graphs.StepGraphs), opt-in with FDDM_STEP_GRAPH=1: bf16 on a GPU
    with the fused optimizer and its grad arena, no GradScaler, one process (the DP all-reduce is issued from
    backward callbacks and stays eager). Off by default: on this ROCm 7 / torch 2.10 stack a replayed step ran 12.9
    ms against 9.94 eager at C2 (tools/ab_graph.sh; the graph launch runs ~1.3 ms longer on the GPU than the same
    launches enqueued eagerly and no longer overlaps the encoder's side stream; DEBUG_CLR_GRAPH_PACKET_CAPTURE and
    DEBUG_HIP_FORCE_GRAPH_QUEUES did not change that) — it pays only where the host, not the GPU, bounds the step.
    Fixed batch shapes only (StepGraphs: a new shape drops the graphs and runs eagerly).

    Refused under DEBUG_HIP_FORCE_GRAPH_QUEUES=0: round 4's A/B arm that differed from its neighbours only by that
    setting died with SIGFPE (gpurun_out/ab_g.log: bash reports `Floating point exception` for bench.py; its stderr
    holds no Python traceback, so the signal came from native code). Hypothesis, not verified: SIGFPE on x86 is an
    integer divide by zero, and if the HIP runtime spreads a graph's launches over the number of queues that knob
    forces, zero queues would make that count a divisor. Either way the arm is gone from
    tools/ab_graph.sh and this check keeps the graph path off under that setting."""
    if os.environ.get("DEBUG_HIP_FORCE_GRAPH_QUEUES", None) == "0":
        return False
    return (torch.device(device).type == "cuda" and rt.compute_dtype() == torch.bfloat16 and scaler is None and
            arena is not None and hasattr(optimizer, "clip_and_step") and not fdist.dp_active() and
            os.environ.get("FDDM_STEP_GRAPH", "0") == "1")


def _enc_stream(dev):
    s = _ENC_STREAMS.get(dev)
    if s is None:
        s = _ENC_STREAMS[dev] = torch.cuda.Stream(dev)    # stream priorities measured no different (round 2)
    return s


def train_one_epoch(encoder, decoder, s_proj, t_embed, t_proj, scheduler, loader, optimizer, device, cfg,
                    global_step, scaler=None, epoch=1, print_epoch_summary=True, draw_t=None):
    """reference train.py:293-449. `draw_t(B)` (optional) supplies t on the device; default
    torch.randint(1, T+1) like the reference. Loss values stay on the device; the progress line is
    refreshed every log.log_every steps so the step loop does not wait on the GPU."""
    encoder.eval()
    decoder.train()
    s_proj.train()
    t_embed.train()
    t_proj.train()
    pad_id = cfg.data["pad_id"]
    T_total = cfg.diffusion["T"]
    log_every = max(1, int(cfg.log.get("log_every", 50)))
    n_step_fd = cfg.lfd["n_step_fd"]
    tau = cfg.lfd.get("tau", 1.0)
    lambda_off = cfg.lfd["lambda_offdiag"]
    trainable = list(decoder.parameters()) + list(s_proj.parameters()) + list(t_embed.parameters()) + \
        list(t_proj.parameters())
    if getattr(optimizer, "arena", 1) is None:
        # decoder grads live in one flat buffer the kernels accumulate into (fddm_hip.runtime.GradArena)
        opt_ids = set(id(p) for g in optimizer.param_groups for p in g["params"])
        dparams = [p for p in decoder.parameters() if p.requires_grad]
        if all(id(p) in opt_ids for p in dparams):
            order = decoder.grad_ready_order() if hasattr(decoder, "grad_ready_order") else None
            optimizer.use_grad_arena(dparams, order)
    if fdist.dp_active() and not getattr(optimizer, "_fddm_replicas_synced", False):
        # DP replicas start from rank 0's weights (DDP's constructor broadcast): the trainable parameters and the
        # frozen encoder's parameters / buffers (a random-init encoder differs per rank otherwise)
        fdist.broadcast_params(trainable + list(encoder.parameters()) + list(encoder.buffers()) +
                               [b for m in (decoder, s_proj, t_embed, t_proj) for b in m.buffers()])
        optimizer._fddm_replicas_synced = True
    arena = getattr(optimizer, "arena", None)
    if arena is not None and fdist.dp_active() and arena.reducer is None:
        fdist.OverlapReducer(arena)     # gradient all-reduce overlapped with backward
    # DP: L_fd's batch-dim statistics and w_t's batch mean over the GLOBAL batch (additive lfd.sync_batch_stats,
    # SURVEY §8(e)); default: each rank's own batch (documented "local-batch L_fd")
    lfd_group = fdist.default_group() if (fdist.dp_active() and cfg.lfd.get("sync_batch_stats", False)) else None
    pbar = loader
    if tqdm is not None and print_epoch_summary:
        pbar = tqdm(loader, desc=f"Epoch {epoch} [train]", leave=False)
    loss_sum = torch.zeros((), device=device)   # accumulated per step: a replayed graph's loss is a static buffer
    nsteps = 0
    aux = [p for m in (s_proj, t_embed, t_proj) for p in m.parameters() if p.requires_grad]
    if (arena is not None and getattr(optimizer, "aux_arena", 1) is None and aux and
            all(id(p) in set(id(q) for g in optimizer.param_groups for q in g["params"]) for p in aux)):
        optimizer.use_aux_arena(aux)    # L_fd projector grads at fixed addresses (None on KL-only steps)

    def step(c, c_mask, x0, t, xt, fd):
        """train.py:351-423 from the decoder forward to the optimizer step; returns (loss, loss_diff, loss_fd)."""
        x_mask = x0 != pad_id
        logits = decoder(xt, t, c, x_mask=x_mask, c_mask=c_mask)
        loss_diff = scheduler.kl_term(xt, x0, logits, t, x_mask)
        loss = loss_diff
        loss_fd = None
        if fd:
            L = x0.shape[1]
            z_text = t_proj(t_embed(logits))
            z_speech = align_speech(s_proj(c), L)
            w_t = scheduler.w_t(t).mean()
            if lfd_group is not None:
                w_t = fdist.global_mean(w_t, lfd_group)
                loss_fd = lfd_loss(z_speech, z_text, lambda_offdiag=lambda_off, group=lfd_group)
            else:
                loss_fd = lfd_loss(z_speech, z_text, lambda_offdiag=lambda_off)
            loss = loss + tau * w_t * loss_fd
        optimizer.zero_grad(set_to_none=True)
        if fd and hasattr(optimizer, "attach_aux"):
            optimizer.attach_aux()
        if scaler is not None:
            scaler.scale(loss).backward()
            fdist.allreduce_grads(trainable)    # before unscale_: overlapped slices may still be in flight
            scaler.unscale_(optimizer)
            torch.nn.utils.clip_grad_norm_([p for p in trainable if p.grad is not None], max_norm=CLIP_MAX_NORM)
            scaler.step(optimizer)
            scaler.update()
        else:
            loss.backward()
            fused = hasattr(optimizer, "clip_and_step")
            # DP: the fused AdamW averages the all-reduced SUM itself (grad_scale = 1/W, no pass over the gradients)
            t_bwd = _mark_allreduce_tail()
            fdist.allreduce_grads(trainable, average=not fused)
            _mark_allreduce_tail(t_bwd)
            if fused:
                # the step zeroes the gradients it reads (the next zero_grad's 156 MB arena fill folded into AdamW)
                optimizer.clip_and_step(max_norm=CLIP_MAX_NORM, zero_grads=True, grad_scale=1.0 / fdist.world(),
                                        return_norm=False)   # the norm is not used here: no sqrt launch
            else:
                torch.nn.utils.clip_grad_norm_([p for p in trainable if p.grad is not None], max_norm=CLIP_MAX_NORM)
                optimizer.step()
        return loss, loss_diff, loss_fd

    graphs = None
    if _step_graph_ok(device, scaler, optimizer, arena):
        graphs = _STEP_GRAPHS.get(decoder)
        if graphs is None:
            graphs = _STEP_GRAPHS[decoder] = StepGraphs(device)
    for c, c_mask, x0 in _encoded(encoder, pbar, device, optimizer):
        B, L = x0.shape
        t = draw_t(B) if draw_t is not None else torch.randint(1, T_total + 1, (B,), device=device)
        xt = scheduler.sample_q(x0, t)
        fd = global_step % n_step_fd == 0
        # HIP-event probes of decoder launches (bench.py's attention rows) need the eager launches
        if graphs is not None and c_mask is None and not rt.probing_any("decoder."):
            inputs = {"c": c, "x0": x0, "t": t, "xt": xt}
            shapes = tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(inputs.items()))
            step_args = (CLIP_MAX_NORM, 1.0 / fdist.world())    # the clip_and_step values a capture bakes in
            if graphs.get(fd, trainable, optimizer, shapes, step_args) is not None:
                loss, loss_diff, loss_fd = graphs.replay(fd, inputs)
            else:
                # the first step of this kind runs eagerly (creating every cache / table it reads), then the kind is
                # captured for the next one (a capture executes nothing)
                loss, loss_diff, loss_fd = step(c, None, x0, t, xt, fd)
                graphs.capture(fd, lambda c, x0, t, xt: step(c, None, x0, t, xt, fd), inputs, trainable, optimizer,
                               step_args)
        else:
            loss, loss_diff, loss_fd = step(c, c_mask, x0, t, xt, fd)
        loss_sum += loss.detach()
        nsteps += 1
        if tqdm is not None and print_epoch_summary and (global_step % log_every == 0):
            post = {"step": global_step, "loss": f"{float(loss):.3f}", "diff": f"{float(loss_diff):.3f}"}
            if loss_fd is not None:
                post["lfd"] = f"{float(loss_fd):.3f}"
            pbar.set_postfix(post)
        global_step += 1
    global LAST_ENQUEUE_DONE
    LAST_ENQUEUE_DONE = time.perf_counter()     # host finished enqueueing the epoch (bench.py: host-bound check)
    avg = float(loss_sum) / max(1, nsteps)
    if print_epoch_summary:
        logging.info(f"[Summary] Epoch {epoch} Avg Train Loss: {avg:.4f}")
    return global_step, avg


def setup_logging():
    os.makedirs("logs", exist_ok=True)
    ts = datetime.now().strftime("%Y%m%d_%H%M%S")
    logger = logging.getLogger()
    logger.setLevel(logging.INFO)
    logger.handlers.clear()
    fmt = logging.Formatter("%(asctime)s - %(levelname)s - %(message)s")
    for h in (logging.FileHandler(os.path.join("logs", f"train_{ts}.log"), encoding="utf-8"), logging.StreamHandler()):
        h.setFormatter(fmt)
        logger.addHandler(h)


def build_models(cfg: Config, device):
    d_model = cfg.model["d_model"]
    vocab = cfg.data["vocab_size"]
    pad_id = cfg.data["pad_id"]
    encoder = AcousticEncoder(**cfg.model["encoder"], d_model=d_model).to(device)
    decoder = DenoisingTransformerDecoder(vocab_size=vocab, d_model=d_model, nhead=cfg.model["nhead"],
                                          num_layers=cfg.model["num_layers"], dim_ff=cfg.model["dim_ff"],
                                          dropout=cfg.model["dropout"], max_len=1024, pad_id=pad_id).to(device)
    d_proj = cfg.model["projector"]["d_proj"]
    s_proj = SpeechProjector(d_in=d_model, d_proj=d_proj).to(device)
    t_embed = TextEmbedding(vocab=vocab, d_out=d_proj, mode="logits").to(device)
    t_proj = TextProjector(d_in=d_proj, d_proj=d_proj).to(device)
    sched = SchedulerAdapter(DiscreteDiffusionScheduler(K=vocab, T=cfg.diffusion["T"], device=device,
                                                        beta_max=cfg.diffusion["beta_max"]))
    return encoder, decoder, s_proj, t_embed, t_proj, sched


def _tokenizer(cfg, tok_path):
    """SentencePiece (reference train.py:596-598): the .model, or the BPE model rebuilt from the .vocab next to it
    (data_io.load_tokenizer); else the offline vocab.json decoder (models.evaluate.VocabTokenizer)."""
    if tok_path:
        try:
            from data_io import load_tokenizer
            return load_tokenizer(tok_path)
        except (FileNotFoundError, ImportError):
            pass
    from models.evaluate import VocabTokenizer
    vj = cfg.data.get("vocab_json") or os.path.join(os.path.dirname(tok_path or "."), "vocab.json")
    return VocabTokenizer(vj)


def save_checkpoint(path, decoder, s_proj, t_embed, t_proj, step, epoch, raw, optimizer=None, **extra):
    """Reference checkpoint layout (train.py:622-664): decoder / s_proj / t_embed / t_proj state_dicts,
    step, epoch, config. Additive keys for resuming: optimizer (torch AdamW layout), rng seed state."""
    ckpt = {"decoder": decoder.state_dict(), "s_proj": s_proj.state_dict(), "t_embed": t_embed.state_dict(),
            "t_proj": t_proj.state_dict(), "step": step, "epoch": epoch, "config": raw}
    ckpt.update(extra)
    if optimizer is not None:
        ckpt["optimizer"] = optimizer.state_dict()
        ckpt["fddm_seed"] = rt.seed_state()
    torch.save(ckpt, path)


def load_checkpoint(path, decoder, s_proj, t_embed, t_proj, optimizer=None, map_location="cpu"):
    """Loads a reference or MI355X checkpoint (weights only, no pickled code); returns (step, epoch)."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    decoder.load_state_dict(ck["decoder"])
    s_proj.load_state_dict(ck["s_proj"])
    t_embed.load_state_dict(ck["t_embed"])
    t_proj.load_state_dict(ck["t_proj"])
    if optimizer is not None and "optimizer" in ck:
        optimizer.load_state_dict(ck["optimizer"])
    if "fddm_seed" in ck:
        rt.set_seed_state(ck["fddm_seed"])
    rt.clear_cache()
    return int(ck.get("step", 1)), int(ck.get("epoch", 0))


def main():
    ap = argparse.ArgumentParser(description="FDDM-ASR Training Script (MI355X)")
    ap.add_argument("--config", type=str, required=True)
    ap.add_argument("--device", type=str, default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--resume", type=str, default=None, help="checkpoint to resume from (additive option)")
    ap.add_argument("--allow-random-encoder", action="store_true",
                    help="train against a random-init WavLM when model.encoder.wavlm_name does not load weights "
                         "(no network: hub names cannot be fetched)")
    args = ap.parse_args()
    setup_logging()
    with open(args.config, "r", encoding="utf-8") as f:
        raw = yaml.safe_load(f)
    cfg = Config(**raw)
    random.seed(cfg.seed)
    torch.manual_seed(cfg.seed)
    rt.reseed(cfg.seed)
    rt.set_precision(cfg.optim.get("precision", "bf16"))
    device = torch.device(args.device)
    if device.type != "cuda":
        raise RuntimeError("the MI355X build runs on a HIP device only (no CPU fallback)")
    distributed = int(os.environ.get("WORLD_SIZE", "1")) > 1
    import torch.distributed as tdist
    if distributed:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        device = torch.device("cuda", local)
        torch.cuda.set_device(device)
        from datetime import timedelta
        tdist.init_process_group("nccl", device_id=device,
                                 timeout=timedelta(seconds=int(os.environ.get("FDDM_DIST_TIMEOUT_S", "1800"))))
        rt.reseed(cfg.seed + tdist.get_rank())
    rank0 = not distributed or int(os.environ.get("RANK", "0")) == 0
    encoder, decoder, s_proj, t_embed, t_proj, sched = build_models(cfg, device)
    if getattr(encoder.backbone, "random_init", False) and not args.allow_random_encoder:
        raise RuntimeError(f"model.encoder.wavlm_name={cfg.model['encoder'].get('wavlm_name')!r} loaded no weights "
                           "(hub names need a network; give a local HF WavLM directory), so the frozen encoder would "
                           "be random; pass --allow-random-encoder to train against it anyway")
    params = list(decoder.parameters()) + list(s_proj.parameters()) + list(t_embed.parameters()) + \
        list(t_proj.parameters())
    optim = FusedAdamW(params, lr=cfg.optim["lr"], weight_decay=cfg.optim["weight_decay"])

    from data_io import CVZhTWDataset  # real-data input path (WAV reader + SentencePiece)
    train_json = cfg.data.get("train_json", "data/processed/train.json")
    val_json = cfg.data.get("val_json", "data/processed/validation.json")    # reference train.py:555
    test_json = cfg.data.get("test_json", "data/processed/test.json")
    tok_path = cfg.data.get("tokenizer_model_path", "data/tokenizer/zh-TW_A/spm_zhTW_A.model")

    def _loader(path, shuffle):
        ds = CVZhTWDataset(path, tok_path, cfg.data.get("max_len", 128), cfg.data["pad_id"], cfg.data.get("bos_id"),
                           cfg.data.get("eos_id"))
        sampler = None
        if distributed and shuffle:
            sampler = torch.utils.data.distributed.DistributedSampler(ds, shuffle=True, drop_last=True)
        return torch.utils.data.DataLoader(ds, batch_size=cfg.optim["batch_size"], shuffle=shuffle and sampler is None,
                                           sampler=sampler, drop_last=shuffle)

    train_loader = _loader(train_json, True)
    val_loader = _loader(val_json, False) if os.path.exists(val_json) else None
    test_loader = _loader(test_json, False) if os.path.exists(test_json) else None
    for what, path, ld in (("validation", val_json, val_loader), ("test", test_json, test_loader)):
        if ld is None:
            logging.warning(f"{what} manifest {path!r} not found: {what} evaluation is skipped")
    tokenizer = _tokenizer(cfg, tok_path) if (val_loader or test_loader) else None
    os.makedirs(cfg.log["ckpt_dir"], exist_ok=True)
    global_step, start_epoch = 1, 1
    if args.resume:
        global_step, last_epoch = load_checkpoint(args.resume, decoder, s_proj, t_embed, t_proj, optim, device)
        start_epoch = last_epoch + 1
    from models.evaluate import evaluate_cer_with_jumpy_sampling, evaluate_validation_loss
    best_val_cer, best_epoch = float("inf"), 0
    for epoch in range(start_epoch, cfg.optim["num_epochs"] + 1):
        logging.info(f"Epoch {epoch}")
        if hasattr(train_loader.sampler, "set_epoch"):
            train_loader.sampler.set_epoch(epoch)
        global_step, train_loss = train_one_epoch(encoder, decoder, s_proj, t_embed, t_proj, sched, train_loader,
                                                  optim, device, cfg, global_step, None, epoch)
        msg = f"[Epoch {epoch} Summary] train_loss={train_loss:.4f}"
        if rank0 and val_loader is not None:
            val_cer = evaluate_cer_with_jumpy_sampling(encoder, decoder, sched, val_loader, device, cfg, tokenizer)
            val_loss = evaluate_validation_loss(encoder, decoder, s_proj, t_embed, t_proj, sched, val_loader, device,
                                                cfg)
            msg += f" | val_loss={val_loss:.4f} | val_cer={val_cer:.4f}"
            if val_cer < best_val_cer:
                best_val_cer, best_epoch = val_cer, epoch
                save_checkpoint(os.path.join(cfg.log["ckpt_dir"], "best_model.pt"), decoder, s_proj, t_embed, t_proj,
                                global_step, epoch, raw, best_val_cer=best_val_cer)
        if rank0 and test_loader is not None:
            test_cer = evaluate_cer_with_jumpy_sampling(encoder, decoder, sched, test_loader, device, cfg, tokenizer)
            msg += f" | test_cer={test_cer:.4f}"
        logging.info(msg)
        if rank0:
            save_checkpoint(os.path.join(cfg.log["ckpt_dir"], f"ep{epoch:03d}.pt"), decoder, s_proj, t_embed, t_proj,
                            global_step, epoch, raw, optimizer=optim)
        if distributed:
            tdist.barrier()     # the other ranks wait here, not inside the next epoch's first all-reduce
    if rank0:
        logging.info(f"Best validation CER: {best_val_cer:.4f} (Epoch {best_epoch})")
    if distributed:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
