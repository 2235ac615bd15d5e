"""Runs the train step's attention launches (WavLM forward, decoder self / cross forward + backward at C2, bf16)
a few times each, for rocprofv3 counter passes (tools/pmc_generic.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
cases = [(32, 12, 499, 499, True, 0.0, False), (32, 8, 256, 256, False, 0.1, True), (32, 8, 256, 499, False, 0.1, False)]
for B, H, Lq, Lk, rel, p, kpm in cases:
    q = torch.randn(B * Lq, H * 64, device=dev, dtype=bf)
    k = torch.randn(B * Lk, H * 64, device=dev, dtype=bf)
    v = torch.randn(B * Lk, H * 64, device=dev, dtype=bf)
    o = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
    lse = torch.empty(B * H, Lq, device=dev)
    gate = torch.rand(B * H, Lq, device=dev) if rel else None
    table = torch.randn(H, 2 * Lk - 1, device=dev) if rel else None
    keep = None
    if kpm:
        keep = torch.ones(B, Lk, dtype=torch.uint8, device=dev)
        keep[:, Lk * 3 // 4:] = 0
    db = ops.drop_bits(B, H, Lq, Lk, dev) if p > 0 else None
    for _ in range(4):
        ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, key_keep=keep, gate=gate, table=table, drop_p=p, seed=1,
                     rng_stream=1, dbits=db)
    if not rel:
        do = torch.randn_like(o)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        for _ in range(4):
            ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, key_keep=keep, drop_p=p, seed=1,
                         rng_stream=1, dbits=db)
torch.cuda.synchronize()
print("ok")
