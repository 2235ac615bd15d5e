"""WavLM attention forward at the C2 encoder shape (B 32, H 12, 499 x 499, gated relative-position bias), HIP-event
timing of 20 launches after 5 warm-ups: the default kernel (round 6: fwd7's bias build, csrc/attn7.hip REL) and the
round-2 fwd5 (fddm_attn_set_kernels(5)).  python tools/wavlm_attn_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
B, H, L = 32, 12, 499
g = torch.Generator(device=dev).manual_seed(0)
q, k, v = (torch.randn(B * L, H * 64, device=dev, dtype=torch.bfloat16, generator=g) for _ in range(3))
o = torch.empty_like(q)
lse = torch.empty(B * H, L, device=dev)
gate = torch.rand(B * H, L, device=dev, generator=g)
table = torch.randn(H, 2 * L - 1, device=dev, generator=g)
fn = lambda: ops.attn_fwd(q, k, v, o, lse, B, H, L, L, gate=gate, table=table)  # noqa: E731
for rnd in range(2):
    for fam in ("auto", "relfwd5"):
        old = ops.attn_force_kernels(fam)
        for _ in range(5):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        ops.attn_force_kernels(old)
        us = s.elapsed_time(e) / 20 * 1e3
        print(f"[{fam:7s}] WavLM attention fwd B{B} H{H} {L}x{L}: {us:.1f} us  "
              f"{4 * L * L * 64 * B * H / us / 1e6:.0f} TFLOP/s", flush=True)
