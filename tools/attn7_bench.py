"""Decoder attention at the C2 / C4 shapes, both kernel families (HIP-event timing, bf16, keep bits written ahead by
the producer as the decoder does): "v6" = attention.hip's 16x16x32 kernels (fwd6, bwd3s / dq4 + dkv4), "auto" = the
default choice (attn7.hip's 32x32x16 kernels where they apply). Prints us per launch and the fraction of the dense
bf16 MFMA peak (fwd 4 Lq Lk 64, bwd 10 Lq Lk 64 FLOP per (b, h)), and the max |difference| between the families'
outputs (bf16 roundings of the same math).
  python tools/attn7_bench.py [iters] [family,family]   (default families: v6,auto; "fwd7" / "fwd8" = the default with
  every forward on the one-chain fwd7 / the two-chain fwd8)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
PEAK = 2500.0


def timeit(fn, iters):
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
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    fams = tuple(sys.argv[2].split(",")) if len(sys.argv) > 2 else ("v6", "auto")
    cases = [("C2 self  L256 B32 H8 kpm", 32, 8, 256, 256, True),
             ("C2 cross 256x499 B32 H8", 32, 8, 256, 499, False),
             ("C4 self  L512 B16 H12 kpm", 16, 12, 512, 512, True),
             ("C4 cross 512x499 B16 H12", 16, 12, 512, 499, False)]
    for name, B, H, Lq, Lk, kpm in cases:
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
        k = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
        v = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
        do = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
        keep = None
        if kpm:   # per-utterance lengths U{L/2..L} as in the bench
            lens = torch.randint(Lk // 2, Lk + 1, (B,), device=dev, generator=g)
            keep = (torch.arange(Lk, device=dev)[None] < lens[:, None]).to(torch.uint8).contiguous()
        fl = 4.0 * B * H * Lq * Lk * 64
        db = ops.drop_bits(B, H, Lq, Lk, dev)
        res, outs = [], {}
        for fam in fams:
            old = ops.attn_force_kernels(fam)
            try:
                ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0)   # the family's storage layout
                tp = timeit(lambda: ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0), iters)
                o = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
                lse = torch.empty(B * H, Lq, device=dev)
                tf = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, key_keep=keep, drop_p=0.1, seed=1,
                                                 rng_stream=1, dbits=db, bits_ready=True), iters)
                dq = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
                dk = torch.empty(B * Lk, H * 64, device=dev, dtype=bf)
                dv = torch.empty(B * Lk, H * 64, device=dev, dtype=bf)
                tb = timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, key_keep=keep,
                                                 drop_p=0.1, seed=1, rng_stream=1, dbits=db), iters)
                outs[fam] = [x.float() for x in (o, dq, dk, dv)]
            finally:
                ops.attn_force_kernels(old)
            res.append(f"{fam}: fwd {tf*1e3:6.1f} us {fl/tf/1e12*1e3/PEAK:5.3f}  bwd {tb*1e3:6.1f} us "
                       f"{2.5*fl/tb/1e12*1e3/PEAK:5.3f}  bits {tp*1e3:5.1f} us")
        diff = [(a_ - b_).abs().max().item() for a_, b_ in zip(outs[fams[0]], outs[fams[-1]])]
        print(f"{name:28s} " + " | ".join(res) + " | max|diff| o/dq/dk/dv " + " ".join(f"{d:.3g}" for d in diff),
              flush=True)


if __name__ == "__main__":
    main()
