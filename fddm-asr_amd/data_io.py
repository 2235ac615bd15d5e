"""Real-data input path (reference train.py:86-161, CVZhTWDataset) — OUT OF the benchmarked hot
path: needs librosa and a SentencePiece model, neither present offline."""
from __future__ import annotations

import json
import os

import torch
from torch.utils.data import Dataset


class CVZhTWDataset(Dataset):
    def __init__(self, json_file, tokenizer_vocab_path, max_len, pad_id, bos_id=None, eos_id=None):
        import sentencepiece as spm
        with open(json_file, "r", encoding="utf-8") as f:
            self.data = json.load(f)
        self.max_len, self.pad_id, self.bos_id, self.eos_id = max_len, pad_id, bos_id, eos_id
        self.tokenizer = spm.SentencePieceProcessor()
        self.tokenizer.load(tokenizer_vocab_path)
        self.max_audio_samples = 20 * 16000
        self.valid = [i for i, it in enumerate(self.data) if it.get("processed_path") and os.path.exists(it["processed_path"])]

    def __len__(self):
        return len(self.valid)

    def __getitem__(self, idx):
        import librosa
        item = self.data[self.valid[idx]]
        wav, _ = librosa.load(item["processed_path"], sr=16000)
        wav = torch.tensor(wav[: self.max_audio_samples], dtype=torch.float32)
        if wav.numel() < self.max_audio_samples:
            wav = torch.cat([wav, torch.zeros(self.max_audio_samples - wav.numel())])
        toks = self.tokenizer.encode(item["normalized_sentence"])
        if self.bos_id is not None:
            toks = [self.bos_id] + toks
        if self.eos_id is not None:
            toks = toks + [self.eos_id]
        toks = toks[: self.max_len] + [self.pad_id] * max(0, self.max_len - len(toks))
        return wav, torch.tensor(toks, dtype=torch.long)
