"""Eager encoder vs the graph-replayed encoder (fddm_hip.graphs) on alternating slots, both precisions, with and
without encoder.proj."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fddm_hip import runtime as rt  # noqa: E402
from fddm_hip.graphs import GraphedEncoder  # noqa: E402

dev = torch.device("cuda:0")
from test_gpu_models import _encoder  # noqa: E402
from helpers import SMALL_WAVLM  # noqa: E402

for prec in ("fp32", "bf16"):
    for geom, d in ((SMALL_WAVLM, 128), ({}, 512), ({}, 768)):
        with rt.use_precision(prec):
            enc = _encoder(geom, d)
            ge = GraphedEncoder(enc)
            g = torch.Generator().manual_seed(1)
            waves = [0.1 * torch.randn(2, 16000 * (1 if geom else 4), generator=g).to(dev) for _ in range(4)]
            refs = [enc(w)[0].float().clone() for w in waves]
            outs = []
            for i, w in enumerate(waves):
                outs.append(ge.run(w, i % 2).float().clone())
            torch.cuda.synchronize()
            errs = [float((a - b).abs().max()) for a, b in zip(outs, refs)]
            print(prec, geom.get("hidden_size", 768), d, "max abs diff per batch", errs, flush=True)
