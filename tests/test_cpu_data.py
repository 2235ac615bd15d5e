"""Real-data input path (reference train.py:86-161, CVZhTWDataset) on CPU: the WAV reader against the integer
scaling soundfile/librosa apply to the reference preprocessor's 16 kHz PCM_16 clips, the SentencePiece BPE
tokenizer rebuilt from the reference's `.vocab` (tests/golden/spm_zhTW_A.vocab.gz is that data file, gzipped)
against the reference's vocab.json id table, and the dataset's filtering / padding / special tokens."""
import gzip
import json
import os
import struct
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import data_io  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def _write_wav(path, frames, sr, tag=1, bits=16):
    """frames: [n, ch] array already in the target sample type's integer / float values"""
    n, ch = frames.shape
    if tag == 1 and bits == 24:
        v = frames.astype(np.int32).reshape(-1)
        b = np.stack([(v & 0xFF), (v >> 8) & 0xFF, (v >> 16) & 0xFF], 1).astype(np.uint8).tobytes()
    else:
        dt = {(1, 8): "u1", (1, 16): "<i2", (1, 32): "<i4", (3, 32): "<f4"}[(tag, bits)]
        b = frames.astype(dt).tobytes()
    block = ch * bits // 8
    fmt = struct.pack("<HHIIHH", tag, ch, sr, sr * block, block, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"LIST" + struct.pack("<I", 4) + b"INFO" + \
        b"data" + struct.pack("<I", len(b)) + b
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def test_wav_reader_scaling(tmp_path):
    rng = np.random.default_rng(0)
    x16 = rng.integers(-32768, 32768, size=(4000, 1))
    _write_wav(tmp_path / "a.wav", x16, 16000)
    np.testing.assert_array_equal(data_io.load_wav_16k(str(tmp_path / "a.wav")), (x16[:, 0] / 32768.0).astype(np.float32))
    st = rng.integers(-32768, 32768, size=(3000, 2))
    _write_wav(tmp_path / "s.wav", st, 16000)
    exp = ((st / 32768.0).astype(np.float32)).mean(axis=1, dtype=np.float32)
    np.testing.assert_array_equal(data_io.load_wav_16k(str(tmp_path / "s.wav")), exp)
    x24 = rng.integers(-(1 << 23), 1 << 23, size=(500, 1))
    _write_wav(tmp_path / "c.wav", x24, 16000, bits=24)
    np.testing.assert_array_equal(data_io.load_wav_16k(str(tmp_path / "c.wav")), (x24[:, 0] / float(1 << 23)).astype(np.float32))
    xf = rng.standard_normal((700, 1)).astype(np.float32) * 0.3
    _write_wav(tmp_path / "f.wav", xf, 16000, tag=3, bits=32)
    np.testing.assert_array_equal(data_io.load_wav_16k(str(tmp_path / "f.wav")), xf[:, 0])
    x8 = rng.integers(0, 256, size=(200, 1))
    _write_wav(tmp_path / "u.wav", x8, 16000, bits=8)
    np.testing.assert_array_equal(data_io.load_wav_16k(str(tmp_path / "u.wav")), ((x8[:, 0] - 128.0) / 128.0).astype(np.float32))


def test_wav_reader_resamples_other_rates(tmp_path):
    t = np.arange(8000) / 8000.0
    tone = (np.sin(2 * np.pi * 440 * t) * 12000).astype(np.int64)[:, None]
    _write_wav(tmp_path / "r.wav", tone, 8000)
    y = data_io.load_wav_16k(str(tmp_path / "r.wav"))
    assert y.shape == (16000,) and y.dtype == np.float32
    ref = np.sin(2 * np.pi * 440 * np.arange(16000) / 16000.0) * 12000 / 32768.0
    assert np.abs(y[200:-200] - ref[200:-200]).max() < 2e-3


@pytest.fixture(scope="module")
def spm_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("tok")
    with gzip.open(os.path.join(GOLD, "spm_zhTW_A.vocab.gz")) as f:
        (d / "spm_zhTW_A.vocab").write_bytes(f.read())
    return d


def test_tokenizer_rebuilt_from_vocab_matches_reference_id_table(spm_dir):
    tok = data_io.load_tokenizer(str(spm_dir / "spm_zhTW_A.model"))     # .model absent -> rebuilt from .vocab
    with gzip.open(os.path.join(GOLD, "vocab_zhTW_A.json.gz")) as f:
        id2tok = json.load(f)["id2token"]
    assert tok.get_piece_size() == len(id2tok) == 8000
    assert [tok.id_to_piece(i) for i in range(8000)] == id2tok
    assert (tok.unk_id(), tok.bos_id(), tok.eos_id(), tok.pad_id()) == (0, 1, 2, 3)
    # whole-word pieces of the reference vocabulary come out as single ids; every piece round-trips
    assert tok.encode("高雄市") == [id2tok.index("▁高雄市")]
    assert [tok.id_to_piece(i) for i in tok.encode("台北捷運交流道")] == ["▁台北捷運", "交流道"]
    for s in ["我們今天去高雄", "政府需要討論這個問題", "台中市的公車系統"]:
        ids = tok.encode(s)
        assert tok.decode(ids) == s and 0 not in ids
        assert "".join(tok.id_to_piece(i) for i in ids) == "▁" + s


def test_dataset_items(tmp_path, spm_dir, monkeypatch):
    monkeypatch.chdir(tmp_path)                     # processed_path is relative to the working directory
    os.makedirs("clips")
    rng = np.random.default_rng(1)
    short = rng.integers(-20000, 20000, size=(16000 * 3, 1))
    long_ = rng.integers(-20000, 20000, size=(16000 * 21, 1))
    _write_wav("clips/a.wav", short, 16000)
    _write_wav("clips/b.wav", long_, 16000)
    items = [{"processed_path": "clips/a.wav", "normalized_sentence": "我們今天去高雄"},
             {"processed_path": "clips/missing.wav", "normalized_sentence": "不"},
             {"processed_path": "clips/b.wav", "normalized_sentence": "交流道" * 40},
             {"normalized_sentence": "沒有音檔"}]
    with open("m.json", "w", encoding="utf-8") as f:
        json.dump(items, f, ensure_ascii=False)
    ds = data_io.CVZhTWDataset("m.json", str(spm_dir / "spm_zhTW_A.model"), max_len=16, pad_id=3, bos_id=1, eos_id=2)
    assert len(ds) == 2
    wav, x0 = ds[0]
    assert wav.shape == (320000,) and wav.dtype == torch.float32
    assert torch.equal(wav[:48000], torch.from_numpy((short[:, 0] / 32768.0).astype(np.float32)))
    assert bool((wav[48000:] == 0).all())
    assert x0.tolist()[:6] == [1, 18, 63, 5140, 1004, 2] and x0.tolist()[6:] == [3] * 10
    wav, x0 = ds[1]
    assert wav.shape == (320000,)
    assert torch.equal(wav, torch.from_numpy((long_[:320000, 0] / 32768.0).astype(np.float32)))
    assert x0.shape == (16,) and x0[0] == 1 and 2 not in x0.tolist() and 3 not in x0.tolist()   # truncated: no eos/pad
    dl = torch.utils.data.DataLoader(ds, batch_size=2)
    w, x = next(iter(dl))
    assert w.shape == (2, 320000) and x.shape == (2, 16)
