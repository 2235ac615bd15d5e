"""CER / WER evaluation (drop-in for models/evaluate.py of the reference).

Same function names and signatures as the reference (_ids_to_text_one, logits_to_text, calculate_cer,
calculate_wer, evaluate_validation_loss, evaluate_cer_with_full_sampling,
evaluate_cer_with_jumpy_sampling, evaluate_wer_with_jumpy_sampling, evaluate_cer_with_multi_sample).
Sampling runs the MI355X jumpy sampler (sampler/jumpy_sampler.py, HIP-graph replay); the edit
distances are the reference's Levenshtein recurrences evaluated one DP row per numpy step.

Deviations: the reference reads the inference section with `cfg.get(...)`, which raises
AttributeError on the train.py Config dataclass (evaluate.py:469-475); here both a dict and the
dataclass are accepted. `VocabTokenizer` decodes ids offline from the tokenizer's vocab.json (the
SentencePiece .model is not shipped with the reference).
"""
from __future__ import annotations

import gzip
import json
from typing import List

import numpy as np
import torch

try:
    from tqdm import tqdm
except Exception:  # pragma: no cover
    tqdm = None


class VocabTokenizer:
    """SentencePiece DecodeIds from vocab.json `id2token` (data/tokenizer/zh-TW_A/vocab.json): pieces
    are concatenated, '▁' becomes a space and the leading space is dropped; <s>, </s>, <pad> decode to
    nothing and <unk> to ' ⁇ ' (SentencePiece's unk surface)."""

    def __init__(self, path_or_dict):
        if isinstance(path_or_dict, dict):
            d = path_or_dict
        else:
            op = gzip.open if str(path_or_dict).endswith(".gz") else open
            with op(path_or_dict, "rt", encoding="utf-8") as f:
                d = json.load(f)
        self.id2token = list(d["id2token"])
        sp = d.get("special_token_ids", {})
        self.unk_id = sp.get("unk_id", 0)
        self.control = {sp.get(k) for k in ("bos_id", "eos_id", "pad_id") if sp.get(k) is not None}

    def DecodeIds(self, ids) -> str:
        out = []
        for i in ids:
            i = int(i)
            if i in self.control:
                continue
            out.append(" ⁇ " if i == self.unk_id else self.id2token[i].replace("▁", " "))
        s = "".join(out)
        return s[1:] if s.startswith(" ") else s

    decode = DecodeIds


def _iter_with_progress(iterable, desc: str, total=None):
    if tqdm is not None:
        try:
            return tqdm(iterable, desc=desc, total=total, leave=False)
        except Exception:
            return tqdm(iterable, desc=desc, leave=False)
    print(desc, flush=True)
    return iterable


def _ids_to_text_one(ids_tensor: torch.Tensor, tokenizer, pad_id: int, bos_id: int | None = None,
                     eos_id: int | None = None) -> str:
    """evaluate.py:26-69: drop pad (and bos), stop at eos, DecodeIds."""
    clean: List[int] = []
    for tid in ids_tensor.detach().to("cpu").tolist():
        if tid == pad_id:
            continue
        if bos_id is not None and tid == bos_id:
            continue
        if eos_id is not None and tid == eos_id:
            break
        clean.append(int(tid))
    try:
        return tokenizer.DecodeIds(clean)
    except Exception:
        try:
            return tokenizer.decode(clean)
        except Exception:
            return tokenizer.Decode(clean)


def logits_to_text(logits: torch.Tensor, tokenizer, pad_id: int, bos_id: int | None = None,
                   eos_id: int | None = None) -> List[str]:
    """evaluate.py:71-91."""
    pred = torch.argmax(logits, dim=-1)
    return [_ids_to_text_one(pred[i], tokenizer, pad_id, bos_id, eos_id) for i in range(pred.size(0))]


def _levenshtein(r, h) -> int:
    """dp[i][j] = min(dp[i-1][j]+1, dp[i][j-1]+1, dp[i-1][j-1]+[r_i≠h_j]) (evaluate.py:101-113), one row
    per step: the deletion/substitution terms are elementwise; the insertion chain dp[i][j-1]+1 is a
    running minimum of (row[j] - j) + j."""
    n = len(h)
    j = np.arange(n + 1, dtype=np.int64)
    prev = j.copy()
    for i in range(1, len(r) + 1):
        cost = (h != r[i - 1]).astype(np.int64)
        row = np.empty(n + 1, dtype=np.int64)
        row[0] = i
        row[1:] = np.minimum(prev[1:] + 1, prev[:-1] + cost)
        prev = np.minimum.accumulate(row - j) + j
    return int(prev[n])


def _codes(s: str) -> np.ndarray:
    return np.frombuffer(s.encode("utf-32-le"), dtype=np.uint32)


def calculate_cer(ref: str, hyp: str) -> float:
    """evaluate.py:93-117 (character Levenshtein / len(ref); empty ref → 0 or 1)."""
    r, h = _codes(ref), _codes(hyp)
    if len(r) == 0:
        return 0.0 if len(h) == 0 else 1.0
    return float(_levenshtein(r, h)) / float(len(r))


def calculate_wer(ref: str, hyp: str) -> float:
    """evaluate.py:119-134 (whitespace words)."""
    rw, hw = ref.strip().split(), hyp.strip().split()
    if len(rw) == 0:
        return 0.0
    vocab = {w: k for k, w in enumerate(dict.fromkeys(rw + hw))}
    r = np.array([vocab[w] for w in rw], dtype=np.int64)
    h = np.array([vocab[w] for w in hw], dtype=np.int64)
    return float(_levenshtein(r, h)) / float(len(r))


def _inference_cfg(cfg) -> dict:
    if hasattr(cfg, "get"):
        return cfg.get("inference", {}) or {}
    return getattr(cfg, "inference", {}) or {}


def _sampler(scheduler, decoder, cfg, device, T_infer, r, greedy, posterior_mode, sampling_mode, temperature):
    from sampler.jumpy_sampler import DiffusionJumpySampler
    return DiffusionJumpySampler(scheduler=scheduler.sch if hasattr(scheduler, "sch") else scheduler, decoder=decoder,
                                 K=cfg.data["vocab_size"], T_train=cfg.diffusion["T"], T_infer=T_infer, r=r,
                                 greedy=greedy, posterior_mode=posterior_mode, sampling_mode=sampling_mode,
                                 temperature=temperature, device=device)


@torch.no_grad()
def evaluate_validation_loss(encoder, decoder, s_proj, t_embed, t_proj, scheduler, data_loader, device, cfg) -> float:
    """evaluate.py:188-246: KL at t = 1 with x_t = x_0, averaged per utterance."""
    for m in (encoder, decoder, s_proj, t_embed, t_proj):
        m.eval()
    pad_id = cfg.data["pad_id"]
    total = torch.zeros((), device=device)
    n = 0
    for wave, x0 in data_loader:
        wave, x0 = wave.to(device), x0.to(device)
        B = x0.shape[0]
        c, c_mask, _ = encoder(wave)
        t = torch.ones(B, dtype=torch.long, device=device)
        xt = x0.clone()
        x_mask = x0 != pad_id
        logits = decoder(xt, t, c, x_mask=x_mask, c_mask=c_mask)
        total += scheduler.kl_term(xt, x0, logits, t, x_mask) * B
        n += B
    return float(total) / n if n else 0.0


@torch.no_grad()
def evaluate_cer_with_full_sampling(encoder, decoder, scheduler, data_loader, device, cfg, tokenizer,
                                    sampling_config: dict | None = None) -> float:
    """evaluate.py:248-350."""
    sc = sampling_config or {}
    inf = _inference_cfg(cfg)
    smp = _sampler(scheduler, decoder, cfg, device, sc.get("T_infer", inf.get("T_infer", 20)), sc.get("r", inf.get("r", 5)),
                   sc.get("greedy", inf.get("greedy", True)), sc.get("posterior_mode", inf.get("posterior_mode", "map")),
                   sc.get("sampling_mode", inf.get("sampling_mode", "exact")),
                   sc.get("temperature", inf.get("temperature", 1.0)))
    encoder.eval()
    decoder.eval()
    pad_id, bos, eos = cfg.data["pad_id"], cfg.data.get("bos_id"), cfg.data.get("eos_id")
    total, n = 0.0, 0
    for wave, x0 in data_loader:
        wave = wave.to(device)
        B, L = x0.shape
        c, _, _ = encoder(wave)
        x_pred, _ = smp.sample(cond_c=c, seq_len=L, graph=True, return_probs=False)
        x_pred = x_pred.cpu()
        for i in range(B):
            total += calculate_cer(_ids_to_text_one(x0[i], tokenizer, pad_id, bos, eos),
                                   _ids_to_text_one(x_pred[i], tokenizer, pad_id, bos, eos))
            n += 1
    return total / n if n else 0.0


@torch.no_grad()
def evaluate_cer_with_jumpy_sampling(encoder, decoder, scheduler, data_loader, device, cfg, tokenizer) -> float:
    """evaluate.py:453-477."""
    inf = _inference_cfg(cfg)
    sc = {"T_infer": inf.get("T_infer", 20), "r": inf.get("r", 5), "greedy": inf.get("greedy", True),
          "posterior_mode": inf.get("posterior_mode", "map"), "sampling_mode": inf.get("sampling_mode", "exact"),
          "temperature": inf.get("temperature", 1.0)}
    return evaluate_cer_with_full_sampling(encoder, decoder, scheduler, data_loader, device, cfg, tokenizer, sc)


@torch.no_grad()
def evaluate_wer_with_jumpy_sampling(encoder, decoder, scheduler, data_loader, device, cfg, tokenizer) -> float:
    """evaluate.py:136-186 (greedy MAP, one utterance per sampler call as in the reference — the
    batched call gives the same ids since utterances are independent)."""
    inf = _inference_cfg(cfg)
    smp = _sampler(scheduler, decoder, cfg, device, inf.get("T_infer", 20), inf.get("r", 5), True, "map",
                   inf.get("sampling_mode", "exact"), inf.get("temperature", 1.0))
    encoder.eval()
    decoder.eval()
    pad_id, bos, eos = cfg.data["pad_id"], cfg.data.get("bos_id"), cfg.data.get("eos_id")
    total, n = 0.0, 0
    for wave, x0 in data_loader:
        B, L = x0.shape
        c, _, _ = encoder(wave.to(device))
        x_pred, _ = smp.sample(cond_c=c, seq_len=L, graph=True, return_probs=False)
        x_pred = x_pred.cpu()
        for i in range(B):
            total += calculate_wer(_ids_to_text_one(x0[i], tokenizer, pad_id, bos, eos),
                                   _ids_to_text_one(x_pred[i], tokenizer, pad_id, bos, eos))
            n += 1
    return total / n if n else 0.0


@torch.no_grad()
def evaluate_cer_with_multi_sample(encoder, decoder, scheduler, data_loader, device, cfg, tokenizer,
                                   sampling_config: dict = None, num_samples: int = 3) -> float:
    """evaluate.py:352-451: per utterance `num_samples` non-greedy draws, of which (as in the
    reference) the first is scored."""
    inf = _inference_cfg(cfg)
    sc = sampling_config or {"T_infer": inf.get("T_infer", 20), "r": inf.get("r", 2),
                             "posterior_mode": inf.get("posterior_mode", "average"),
                             "sampling_mode": inf.get("sampling_mode", "exact"),
                             "temperature": inf.get("temperature", 1.0)}
    smp = _sampler(scheduler, decoder, cfg, device, sc["T_infer"], sc["r"], False, sc["posterior_mode"],
                   sc["sampling_mode"], sc["temperature"])
    encoder.eval()
    decoder.eval()
    pad_id, bos, eos = cfg.data["pad_id"], cfg.data.get("bos_id"), cfg.data.get("eos_id")
    total, n = 0.0, 0
    for wave, x0 in data_loader:
        B, L = x0.shape
        c, _, _ = encoder(wave.to(device))
        draws = [smp.sample(cond_c=c, seq_len=L, return_probs=False)[0].cpu() for _ in range(num_samples)]
        for i in range(B):
            total += calculate_cer(_ids_to_text_one(x0[i], tokenizer, pad_id, bos, eos),
                                   _ids_to_text_one(draws[0][i], tokenizer, pad_id, bos, eos))
            n += 1
    return total / n if n else 0.0
