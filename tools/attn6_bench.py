"""Decoder attention forward at the C2 / C4 shapes: fwd6 (streamed ring, precomputed dropout bits; NG 1 / 2) vs fwd3
(K/V resident, FDDM_ATTN_FWD6=0), and the dropout-bit producer alone. HIP-event timing, bf16. Also checks that fwd6
and fwd3 give bit-identical outputs, lse and keep-bit words.
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
        outs = {}
        res = []
        for tag, env, ready in (("fwd3", {"FDDM_ATTN_FWD6": "0"}, False), ("fwd6 words/ng2", {"FDDM_ATTN_NG6": "2"}, True),
                                ("fwd6 tables/ng1", {"FDDM_ATTN_NG6": "1"}, False),
                                ("fwd6 tables/ng2", {"FDDM_ATTN_NG6": "2"}, False)):
            o = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
            lse = torch.empty(B * H, Lq, device=dev)
            db = ops.drop_bits(B, H, Lq, Lk, dev)
            os.environ.update(env)
            if ready:
                ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0)
            f = lambda: ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, key_keep=keep, drop_p=0.1, seed=1,  # noqa
                                     rng_stream=1, dbits=db, bits_ready=ready)
            t = timeit(f)
            for k_ in env:
                del os.environ[k_]
            outs[tag] = (o.clone(), lse.clone(), db.clone())
            res.append(f"{tag} {t*1e3:6.1f} us {fl/t/1e12*1e3/2500:5.3f}")
        tb = timeit(lambda: ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0))
        ref = outs["fwd3"]
        same = []
        for tag in ("fwd6 words/ng2", "fwd6 tables/ng1", "fwd6 tables/ng2"):
            o6, l6, d6 = outs[tag]
            nt = (Lk + 63) // 64
            # words of key tiles that are all padding are not written by fwd3: compare the rest
            same.append(f"{tag}: O {torch.equal(o6, ref[0])} lse {torch.equal(l6, ref[1])}")
        dwords = torch.equal(outs["fwd6 tables/ng2"][2].view(B * H, -1, Lq)[:, :1], ref[2].view(B * H, -1, Lq)[:, :1])
        print(f"{name:28s} " + " | ".join(res) + f" | bits alone {tb*1e3:5.1f} us | " + "; ".join(same) +
              f"; tile-0 words equal {dwords}", flush=True)
        # backward: v2 (dq2 + dkv2), v4 (streamed dq4 + dkv4), fused bwd3s (self L <= 256), on the fwd6 outputs
        o, lse, db = outs["fwd6 tables/ng2"]
        do = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
        grads = {}
        rb = []
        for tag, env in (("v2", {"FDDM_ATTN_BWD4": "0", "FDDM_ATTN_BWD_SPLIT": "1"}), ("v4", {"FDDM_ATTN_BWD4": "2"}),
                         ("default", {})):
            dq = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
            dk = torch.empty(B * Lk, H * 64, device=dev, dtype=bf)
            dv = torch.empty(B * Lk, H * 64, device=dev, dtype=bf)
            os.environ.update(env)
            fb = lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, key_keep=keep, drop_p=0.1,  # noqa
                                      seed=1, rng_stream=1, dbits=db)
            t = timeit(fb)
            for k_ in env:
                del os.environ[k_]
            grads[tag] = (dq.float(), dk.float(), dv.float())
            rb.append(f"{tag} {t*1e3:6.1f} us {2.5*fl/t/1e12*1e3/2500:5.3f}")
        err = [float((x - y).norm() / y.norm()) for x, y in zip(grads["v4"], grads["v2"])]
        print(f"{'  bwd':28s} " + " | ".join(rb) + " | v4 vs v2 rel " + " ".join(f"{e:.1e}" for e in err), flush=True)


if __name__ == "__main__":
    main()
