"""fwd7 alone at the four decoder shapes (keep bits ready), us per launch: python tools/probe/attn7_fwdonly.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402
from attn7_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
out = []
for name, B, H, Lq, Lk, kpm in (("c2self", 32, 8, 256, 256, True), ("c2cross", 32, 8, 256, 499, False),
                                ("c4self", 16, 12, 512, 512, True), ("c4cross", 16, 12, 512, 499, False)):
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
    k = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
    v = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
    keep = None
    if kpm:
        lens = torch.randint(Lk // 2, Lk + 1, (B,), device=dev, generator=g)
        keep = (torch.arange(Lk, device=dev)[None] < lens[:, None]).to(torch.uint8).contiguous()
    db = ops.drop_bits(B, H, Lq, Lk, dev)
    ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0)
    o = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
    lse = torch.empty(B * H, Lq, device=dev)
    t = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, key_keep=keep, drop_p=0.1, seed=1, rng_stream=1,
                                    dbits=db, bits_ready=True), 30)
    t0 = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, key_keep=keep), 30)
    out.append(f"{name} {t*1e3:5.1f} (p=0 {t0*1e3:5.1f})")
print(" | ".join(out), flush=True)
