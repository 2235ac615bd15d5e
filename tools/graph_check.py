"""The train loop's _encoded generator (side stream + graph slots) vs the eager encoder, with main-stream work
between batches that allocates and writes memory like a decoder step would."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fddm_hip import runtime as rt  # noqa: E402
import train as T_  # noqa: E402
from test_gpu_models import _encoder  # noqa: E402
from helpers import SMALL_WAVLM  # noqa: E402

dev = torch.device("cuda:0")


class Opt:
    param_groups = [{"params": []}]


for prec in ("fp32", "bf16"):
    for geom, d, sec in ((SMALL_WAVLM, 128, 1), ({}, 768, 4), ({}, 512, 4)):
        with rt.use_precision(prec):
            enc = _encoder(geom, d)
            g = torch.Generator().manual_seed(1)
            loader = [(0.1 * torch.randn(2, 16000 * sec, generator=g), torch.zeros(2, 8, dtype=torch.long))
                      for _ in range(5)]
            refs = [enc(w.to(dev))[0].float().clone() for w, _ in loader]
            errs_y, errs_e = [], []
            for i, (c, _, _) in enumerate(T_._encoded(enc, loader, dev, Opt())):
                a = c.float().clone()
                junk = [torch.randn(4096, 4096, device=dev) for _ in range(3)]
                for _ in range(4):
                    junk[0] = junk[1] @ junk[2] + junk[0]
                del junk
                b = c.float().clone()
                errs_y.append(float((a - refs[i]).abs().max()))
                errs_e.append(float((b - refs[i]).abs().max()))
            torch.cuda.synchronize()
            print(prec, geom.get("hidden_size", 768), d, "at yield", errs_y, "after step", errs_e, flush=True)
