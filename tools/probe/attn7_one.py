"""One decoder-attention shape, both kernel families, a few launches each (for rocprofv3 counter passes).
  python tools/probe/attn7_one.py [c2self|c2cross|c4self|c4cross] [fwd|bwd|both] [families, default v6,auto]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

SH = {"c2self": (32, 8, 256, 256, True), "c2cross": (32, 8, 256, 499, False), "c4self": (16, 12, 512, 512, True),
      "c4cross": (16, 12, 512, 499, False)}
which = sys.argv[1] if len(sys.argv) > 1 else "c4self"
what = sys.argv[2] if len(sys.argv) > 2 else "both"
B, H, Lq, Lk, kpm = SH[which]
dev = torch.device("cuda:0")
bf = torch.bfloat16
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
k = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
v = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
do = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
keep = None
if kpm:
    lens = torch.randint(Lk // 2, Lk + 1, (B,), device=dev, generator=g)
    keep = (torch.arange(Lk, device=dev)[None] < lens[:, None]).to(torch.uint8).contiguous()
db = ops.drop_bits(B, H, Lq, Lk, dev)
o = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
lse = torch.empty(B * H, Lq, device=dev)
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
for fam in (sys.argv[3] if len(sys.argv) > 3 else "v6,auto").split(","):
    old = ops.attn_force_kernels(fam)
    ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0)
    for _ in range(5):
        ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, key_keep=keep, drop_p=0.1, seed=1, rng_stream=1, dbits=db,
                     bits_ready=True)
        if what != "fwd":
            ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, key_keep=keep, drop_p=0.1, seed=1,
                         rng_stream=1, dbits=db)
    ops.attn_force_kernels(old)
torch.cuda.synchronize()
print("ok")
