"""Decoder attention at the C2 / C4 shapes (HIP-event timing, bf16): the forward (fwd6) with the keep bits written
ahead by the producer (as the decoder runs it) and with the bits drawn in-kernel from LDS tables (what a standalone
attn_fwd call without precomputed bits runs), the producer alone for one site, and the backward (bwd3s / dq4 + dkv4 by
shape). Checks that both forward modes give bit-identical outputs, LSE and keep words. The round-4 comparison against
the removed fwd3 / dq2-dkv2-only paths is in profiles/r04_attn6_bench.txt.
  python tools/attn6_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ops.attn_force_kernels("v6")    # this tool times the round-4 family (keep bits in its word layout)
    cases = [("C2 self  L256 B32 H8 kpm", 32, 8, 256, 256, True),
             ("C2 cross 256x499 B32 H8", 32, 8, 256, 499, False),
             ("C4 self  L512 B16 H12 kpm", 16, 12, 512, 512, True),
             ("C4 cross 512x499 B16 H12", 16, 12, 512, 499, False)]
    for name, B, H, Lq, Lk, kpm in cases:
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
        k = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
        v = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
        keep = None
        if kpm:   # per-utterance lengths U{L/2..L} as in the bench
            lens = torch.randint(Lk // 2, Lk + 1, (B,), device=dev, generator=g)
            keep = (torch.arange(Lk, device=dev)[None] < lens[:, None]).to(torch.uint8).contiguous()
        fl = 4.0 * B * H * Lq * Lk * 64
        outs, res = {}, []
        for tag, ready in (("words", True), ("tables", False)):
            o = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
            lse = torch.empty(B * H, Lq, device=dev)
            db = ops.drop_bits(B, H, Lq, Lk, dev)
            if ready:
                ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0)
            f = lambda: ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, key_keep=keep, drop_p=0.1, seed=1,  # noqa
                                     rng_stream=1, dbits=db, bits_ready=ready)
            t = timeit(f)
            outs[tag] = (o.clone(), lse.clone(), db.clone())
            res.append(f"fwd6 {tag} {t*1e3:6.1f} us {fl/t/1e12*1e3/2500:5.3f}")
        tb = timeit(lambda: ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0))
        ns = 6     # the train step produces all blocks' sites of one kind in one launch
        db6 = torch.empty(ns, db.numel(), device=dev, dtype=torch.int64)
        tb6 = timeit(lambda: ops.attn_drop_bits(db6, ns, B, H, Lq, Lk, 0.1, 1, 1, 6))
        same = all(torch.equal(a_, b_) for a_, b_ in zip(outs["words"][:2], outs["tables"][:2]))
        wsame = torch.equal(outs["words"][2].view(B * H, -1, Lq)[:, :1], outs["tables"][2].view(B * H, -1, Lq)[:, :1])
        o, lse, db = outs["words"]
        do = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
        dq = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
        dk = torch.empty(B * Lk, H * 64, device=dev, dtype=bf)
        dv = torch.empty(B * Lk, H * 64, device=dev, dtype=bf)
        tbw = timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, key_keep=keep, drop_p=0.1,
                                          seed=1, rng_stream=1, dbits=db))
        print(f"{name:28s} " + " | ".join(res) + f" | bits alone {tb*1e3:5.1f} us, x{ns} sites {tb6*1e3/ns:5.1f} us/site | bwd {tbw*1e3:6.1f} us "
              f"{2.5*fl/tbw/1e12*1e3/2500:5.3f} | outputs equal {same}, tile-0 words equal {wsame}", flush=True)


if __name__ == "__main__":
    main()
