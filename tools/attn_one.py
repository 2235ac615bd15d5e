"""Runs one attention configuration a few times (for rocprofv3 counter passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
which = sys.argv[1] if len(sys.argv) > 1 else "wavlm"
B, H, Lq, Lk = (32, 12, 499, 499) if which == "wavlm" else (32, 8, 256, 256)
q = torch.randn(B * Lq, H * 64, device=dev, dtype=torch.bfloat16)
k = torch.randn(B * Lk, H * 64, device=dev, dtype=torch.bfloat16)
v = torch.randn(B * Lk, H * 64, device=dev, dtype=torch.bfloat16)
o = torch.empty_like(q)
lse = torch.empty(B * H, Lq, device=dev)
gate = torch.rand(B * H, Lq, device=dev) if which == "wavlm" else None
table = torch.randn(H, 2 * Lk - 1, device=dev) if which == "wavlm" else None
for _ in range(5):
    ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, gate=gate, table=table)
if which != "wavlm":
    do = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    for _ in range(5):
        ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk)
torch.cuda.synchronize()
print("ok")
