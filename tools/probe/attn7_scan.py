"""fwd7 launch time vs key-range length at fixed queries (C2 / C4 query geometry, dropout bits ready, no mask):
intercept = prologue + epilogue + launch, slope = per 64-key tile.  python tools/probe/attn7_scan.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for (B, H, Lq) in ((32, 8, 256), (16, 12, 512)):
    row = []
    for Lk in (64, 128, 256, 512, 1024):
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
        k = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
        v = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
        db = ops.drop_bits(B, H, Lq, Lk, dev)
        ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0)
        o = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
        lse = torch.empty(B * H, Lq, device=dev)
        for fam in ("auto", "v6"):
            old = ops.attn_force_kernels(fam)
            t = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, drop_p=0.1, seed=1, rng_stream=1, dbits=db,
                                            bits_ready=True))
            ops.attn_force_kernels(old)
            t0 = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, drop_p=0.0)) if fam == "auto" else 0
            row.append(f"Lk {Lk:4d} {fam}: {t:6.1f} us" + (f" (p=0 {t0:6.1f})" if fam == "auto" else ""))
    print(f"B{B} H{H} Lq{Lq}: " + " | ".join(row), flush=True)
