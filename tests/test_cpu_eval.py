"""CER / WER evaluation host logic vs fixtures generated with the reference's
models/evaluate.py (tests/golden/make_golden.py:gen_cer). CPU only."""
import os

import numpy as np
import torch

from conftest import GOLDEN
from helpers import load


def test_cer_wer_match_reference():
    from models.evaluate import calculate_cer, calculate_wer
    g = load("cer")
    for a, b, c, w in zip(g["refs"], g["hyps"], g["cer"], g["wer"]):
        assert calculate_cer(str(a), str(b)) == float(c), (a, b)
        assert calculate_wer(str(a), str(b)) == float(w), (a, b)


def test_ids_to_text_filtering_matches_reference():
    from models.evaluate import _ids_to_text_one

    class Rec:
        def DecodeIds(self, ids):
            return ",".join(str(i) for i in ids)

    g = load("cer")
    ids = torch.from_numpy(g["ids"])
    for i in range(ids.shape[0]):
        got = _ids_to_text_one(ids[i], Rec(), pad_id=0, bos_id=1 if i % 2 else None, eos_id=2 if i % 3 else None)
        assert got == str(g["clean"][i])


def test_vocab_tokenizer_decode_rules():
    """Offline SentencePiece decode from the reference tokenizer's vocab.json (data file copied to
    tests/golden): pieces joined, '▁' -> space, leading space dropped, control ids silent, unk ' ⁇ '.
    Parity with the SentencePiece .model is unpinned (the model file is not shipped)."""
    from models.evaluate import VocabTokenizer, logits_to_text
    tok = VocabTokenizer(os.path.join(GOLDEN, "vocab_zhTW_A.json.gz"))
    assert len(tok.id2token) == 8000
    assert tok.DecodeIds([4, 6]) == "我可以"            # '▁我' '可以'
    assert tok.DecodeIds([4, 5]) == "我 這"             # '▁我' '▁這'
    assert tok.DecodeIds([1, 4, 3, 2]) == "我"
    assert tok.DecodeIds([0, 6]) == "⁇ 可以"
    assert tok.DecodeIds([]) == ""
    logits = torch.zeros(1, 3, 8000)
    logits[0, 0, 4] = logits[0, 1, 6] = logits[0, 2, 3] = 1.0
    assert logits_to_text(logits, tok, pad_id=3) == ["我可以"]
