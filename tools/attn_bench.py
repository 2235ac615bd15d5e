"""Micro-benchmark of libfddm_hip attention at the train step's shapes (HIP-event timing, bf16).
Forward v2 vs v1 (FDDM_ATTN_V1 is read per launch) and the backward pair."""
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
    cases = [("WavLM self S=499 B32 H12 (relbias)", 32, 12, 499, 499, True, 0.0, False),
             ("decoder self L=256 B32 H8 (kpm, drop .1)", 32, 8, 256, 256, False, 0.1, True),
             ("decoder self L=256 B32 H8 (no drop)", 32, 8, 256, 256, False, 0.0, True),
             ("decoder cross 256x499 B32 H8 (drop .1)", 32, 8, 256, 499, False, 0.1, False),
             ("decoder cross, K|V in the 6-block buffer", 32, 8, 256, 499, False, 0.1, False)]
    for name, B, H, Lq, Lk, rel, p, kpm in cases:
        q = torch.randn(B * Lq, H * 64, device=dev, dtype=bf)
        if "6-block" in name:     # block 2's K|V columns of the fused [B*S, 6 * 2d] projection (row stride 6144)
            kv = torch.randn(B * Lk, 6 * 2 * H * 64, device=dev, dtype=bf)
            k, v = kv[:, 2048:2560], kv[:, 2560:3072]
        else:
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
        f = lambda: ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, key_keep=keep, gate=gate, table=table,  # noqa
                                 drop_p=p, seed=1, rng_stream=1, dbits=db)
        fl = 4.0 * B * H * Lq * Lk * 64
        res = []
        envs = (("v3/16w", {}), ("v3/4w", {"FDDM_ATTN_NW": "4"}), ("v3/8w", {"FDDM_ATTN_NW": "8"}),
                ("v2", {"FDDM_ATTN_V2": "1"}))
        if rel:   # the WavLM forward runs fwd2 by default; fwd3 (K/V resident) on request
            envs = (("fwd2", {}), ("fwd3/16w", {"FDDM_ATTN_REL3": "1"}), ("fwd3/8w", {"FDDM_ATTN_REL3": "1", "FDDM_ATTN_NW": "8"}))
        for tag, env in envs:
            os.environ.update(env)
            t = timeit(f)
            for k_ in env:
                del os.environ[k_]
            res.append(f"{tag} {t*1e3:7.1f} us {fl/t/1e9:6.1f} TF/s")
        print(f"fwd {name:44s} " + " | ".join(res), flush=True)
        if not rel:
            do = torch.randn_like(o)
            dq, dk, dv = torch.empty_like(q), torch.empty(B * Lk, H * 64, device=dev, dtype=bf), \
                torch.empty(B * Lk, H * 64, device=dev, dtype=bf)
            g = lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, H, Lq, Lk, key_keep=keep, drop_p=p,  # noqa
                                     seed=1, rng_stream=1, dbits=db)
            tb = timeit(g)
            os.environ["FDDM_ATTN_DQ2"] = "1"
            tq2 = timeit(g)
            os.environ["FDDM_ATTN_DKV2"] = "1"
            tb2 = timeit(g)
            del os.environ["FDDM_ATTN_DQ2"]
            tk2 = timeit(g)
            del os.environ["FDDM_ATTN_DKV2"]
            print(f"bwd {name:44s}    v3 {tb*1e3:6.1f} us {2.5*fl/tb/1e9:6.1f} TF/s | dq2+dkv3 {tq2*1e3:6.1f} | "
                  f"dq3+dkv2 {tk2*1e3:6.1f} | v2 {tb2*1e3:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
