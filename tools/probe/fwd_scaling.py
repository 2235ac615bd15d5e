"""fwd7 at the C2 self geometry (H 8, L 256, key padding, dropout 0.1, keep bits ready) for B = 16 .. 128: time per
launch and per utterance — whether more resident waves per SIMD (B 64: 3 per SIMD at fwd7's 3-workgroup occupancy)
raise throughput, i.e. whether the kernel is latency-bound at C2's 2 waves per SIMD."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "fddm-asr_amd"))
import torch
from fddm_hip import ops
dev = torch.device("cuda:0"); bf = torch.bfloat16
def timeit(fn, iters=50):
    for _ in range(5): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3
H, L = 8, 256
for B in (16, 32, 48, 64, 96, 128):
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B * L, H * 64, device=dev, dtype=bf, generator=g)
    k = torch.randn(B * L, H * 64, device=dev, dtype=bf, generator=g)
    v = torch.randn(B * L, H * 64, device=dev, dtype=bf, generator=g)
    keep = torch.ones(B, L, device=dev, dtype=torch.uint8)
    db = ops.drop_bits(B, H, L, L, dev)
    ops.attn_drop_bits(db.view(1, -1), 1, B, H, L, L, 0.1, 1, 1, 0)
    o = torch.empty_like(q); lse = torch.empty(B * H, L, device=dev)
    us = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, B, H, L, L, key_keep=keep, drop_p=0.1, seed=1, rng_stream=1,
                                     dbits=db, bits_ready=True))
    fl = 4.0 * B * H * L * L * 64
    print(f"B {B:4d}: {us:7.1f} us, {us / B:6.3f} us/utt, {fl / us / 1e6 / 2500:.3f} of peak", flush=True)
