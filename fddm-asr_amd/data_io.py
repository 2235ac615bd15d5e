"""Real-data input path: the reference's `CVZhTWDataset` (train.py:86-161) with the same
constructor, filtering, audio/token padding and item layout, built on what this image has offline.

* Audio. The reference reads `processed_path` with `librosa.load(path, sr=16000)`. Its preprocessor writes those
  clips as 16 kHz mono PCM_16 WAV (scripts/preprocess.py:118-135, `sf.write(..., subtype="PCM_16")`), for which
  librosa returns soundfile's float32 samples unchanged: int16 / 32768. `load_wav_16k` parses the RIFF/WAVE
  container itself (PCM 8/16/24/32-bit, IEEE float 32/64, WAVE_FORMAT_EXTENSIBLE) with the same integer scaling
  and librosa's channel mean for multi-channel files, so those clips load bit-identically. A clip at another rate
  is resampled with a polyphase filter (scipy.signal.resample_poly): librosa's default soxr_hq resampler is not
  in the image, so that case is close to, not identical with, the reference (never produced by its preprocessor).
* Text. `tokenizer.encode(item["normalized_sentence"])` with the SentencePiece model at `tokenizer_vocab_path`.
  When the binary `.model` is absent (the reference ships only `spm_zhTW_A.vocab` + `vocab.json`),
  `load_tokenizer` rebuilds the BPE model from the `.vocab` (piece, score) table — the reference trains it as
  `model_type=bpe`, unk/bos/eos/pad = 0/1/2/3, default nmt_nfkc normalisation (scripts/tokenizer_train.py:91-124,
  configs/tokenizer_zhTW.yaml) — and hands it to SentencePiece's own BPE encoder, so ids and segmentation come from
  the same pieces, scores and normaliser as the reference's model.
"""
from __future__ import annotations

import io
import json
import os
import struct

import numpy as np
import torch
from torch.utils.data import Dataset

TARGET_SR = 16000

_WAVE_PCM, _WAVE_FLOAT, _WAVE_EXT = 1, 3, 0xFFFE


def load_wav_16k(path: str, target_sr: int = TARGET_SR) -> np.ndarray:
    """float32 mono samples of a RIFF/WAVE file at `target_sr` (librosa.load(path, sr=target_sr) for the
    reference's preprocessed clips; see the module docstring)."""
    with open(path, "rb") as f:
        blob = f.read()
    if len(blob) < 12 or blob[:4] != b"RIFF" or blob[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    fmt = data = None
    pos = 12
    while pos + 8 <= len(blob):
        cid, size = blob[pos:pos + 4], struct.unpack_from("<I", blob, pos + 4)[0]
        body = blob[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = body
        elif cid == b"data":
            data = body
        pos += 8 + size + (size & 1)
    if fmt is None or data is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, nch, sr, _, block, bits = struct.unpack_from("<HHIIHH", fmt, 0)
    if tag == _WAVE_EXT and len(fmt) >= 26:
        tag = struct.unpack_from("<H", fmt, 24)[0]     # the sub-format GUID's first two bytes
    width = bits // 8
    n = len(data) // block
    raw = np.frombuffer(data[: n * block], dtype=np.uint8).reshape(n, nch, block // nch)[:, :, :width]
    if tag == _WAVE_PCM:
        if width == 1:
            x = (raw[..., 0].astype(np.float32) - 128.0) / 128.0
        elif width == 2:
            x = raw.copy().view("<i2")[..., 0].astype(np.float32) / 32768.0
        elif width == 3:
            v = raw[..., 0].astype(np.int32) | (raw[..., 1].astype(np.int32) << 8) | (raw[..., 2].astype(np.int32) << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = v.astype(np.float32) / float(1 << 23)
        elif width == 4:
            x = (raw.copy().view("<i4")[..., 0].astype(np.float64) / float(1 << 31)).astype(np.float32)
        else:
            raise ValueError(f"{path}: {bits}-bit PCM is not supported")
    elif tag == _WAVE_FLOAT and width in (4, 8):
        x = raw.copy().view("<f4" if width == 4 else "<f8")[..., 0].astype(np.float32)
    else:
        raise ValueError(f"{path}: WAVE format tag {tag:#x} is not supported")
    x = x.mean(axis=1, dtype=np.float32) if nch > 1 else x[:, 0]   # librosa.to_mono: channel mean
    if sr != target_sr:
        from math import gcd

        from scipy.signal import resample_poly
        g = gcd(sr, target_sr)
        x = resample_poly(x, target_sr // g, sr // g).astype(np.float32)
    return np.ascontiguousarray(x, dtype=np.float32)


def _nmt_nfkc_normalizer():
    """SentencePiece's built-in nmt_nfkc normaliser spec (its precompiled char map), taken from a throwaway
    model trained in memory — the rule the reference's tokenizer was trained with (the trainer's default)."""
    import sentencepiece as spm
    from sentencepiece import sentencepiece_model_pb2 as pb
    w = io.BytesIO()
    spm.SentencePieceTrainer.train(sentence_iterator=iter(["ab cd ef"] * 8), model_writer=w, vocab_size=12,
                                   model_type="bpe", normalization_rule_name="nmt_nfkc", minloglevel=2,
                                   unk_id=0, bos_id=1, eos_id=2, pad_id=3)
    m = pb.ModelProto()
    m.ParseFromString(w.getvalue())
    return m


def spm_model_from_vocab(vocab_path: str) -> bytes:
    """Serialized SentencePiece BPE ModelProto rebuilt from a `.vocab` (piece \\t score per line, id order)."""
    from sentencepiece import sentencepiece_model_pb2 as pb
    base = _nmt_nfkc_normalizer()
    m = pb.ModelProto()
    m.normalizer_spec.CopyFrom(base.normalizer_spec)
    m.trainer_spec.CopyFrom(base.trainer_spec)
    specials = {0: pb.ModelProto.SentencePiece.UNKNOWN, 1: pb.ModelProto.SentencePiece.CONTROL,
                2: pb.ModelProto.SentencePiece.CONTROL, 3: pb.ModelProto.SentencePiece.CONTROL}
    with open(vocab_path, "r", encoding="utf-8") as f:
        for i, line in enumerate(f):
            line = line.rstrip("\n")
            if not line:
                continue
            piece, score = line.split("\t")
            p = m.pieces.add()
            p.piece = piece
            p.score = float(score)
            p.type = specials.get(i, pb.ModelProto.SentencePiece.NORMAL)
    m.trainer_spec.vocab_size = len(m.pieces)
    m.trainer_spec.model_type = pb.TrainerSpec.BPE
    m.trainer_spec.unk_id, m.trainer_spec.bos_id, m.trainer_spec.eos_id, m.trainer_spec.pad_id = 0, 1, 2, 3
    return m.SerializeToString()


def load_tokenizer(model_path: str):
    """SentencePieceProcessor for `model_path` (reference: `spm.SentencePieceProcessor().load(path)`); when only
    the `.vocab` next to it exists, the BPE model rebuilt from it (spm_model_from_vocab)."""
    import sentencepiece as spm
    tok = spm.SentencePieceProcessor()
    if os.path.exists(model_path):
        tok.load(model_path)
        return tok
    vocab = os.path.splitext(model_path)[0] + ".vocab"
    if not os.path.exists(vocab):
        raise FileNotFoundError(f"tokenizer: neither {model_path} nor {vocab} exists")
    tok.LoadFromSerializedProto(spm_model_from_vocab(vocab))
    return tok


class CVZhTWDataset(Dataset):
    """Reference train.py:86-161: items of `json_file` whose `processed_path` exists; each item is (wav float32
    [20 s x 16 kHz], truncated or zero-padded; token ids [max_len] with optional bos/eos, truncated or pad-filled)."""

    def __init__(self, json_file, tokenizer_vocab_path, max_len, pad_id, bos_id=None, eos_id=None):
        super().__init__()
        with open(json_file, "r", encoding="utf-8") as f:
            self.data = json.load(f)
        self.max_len, self.pad_id, self.bos_id, self.eos_id = max_len, pad_id, bos_id, eos_id
        self.tokenizer = load_tokenizer(tokenizer_vocab_path)
        self.max_audio_samples = 20 * TARGET_SR
        self.valid_indices = [i for i, it in enumerate(self.data)
                              if it.get("processed_path") and os.path.exists(it["processed_path"])]

    def __len__(self):
        return len(self.valid_indices)

    def __getitem__(self, idx):
        item = self.data[self.valid_indices[idx]]
        wav = torch.from_numpy(load_wav_16k(item["processed_path"]))
        if wav.numel() > self.max_audio_samples:
            wav = wav[: self.max_audio_samples]
        elif wav.numel() < self.max_audio_samples:
            wav = torch.cat([wav, torch.zeros(self.max_audio_samples - wav.numel())])
        tokens = list(self.tokenizer.encode(item["normalized_sentence"]))
        if self.bos_id is not None:
            tokens = [self.bos_id] + tokens
        if self.eos_id is not None:
            tokens = tokens + [self.eos_id]
        tokens = tokens[: self.max_len] + [self.pad_id] * max(0, self.max_len - len(tokens))
        return wav, torch.tensor(tokens, dtype=torch.long)
