"""Time the bf16 attention kernels at the train step's shapes (HIP events); run per library variant
(FDDM_HIP_LIB) to A/B kernel experiments.   python tools/attn_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16


def main():
    res = []
    g = torch.Generator(device=dev).manual_seed(1)
    # WavLM: B 32, H 12, S 499, gated rel-pos bias, no dropout
    B, H, S = 32, 12, 499
    qkv = torch.randn(B * S, 3 * H * 64, device=dev, dtype=bf, generator=g)
    o = torch.empty(B * S, H * 64, device=dev, dtype=bf)
    lse = torch.empty(B * H, S, device=dev)
    gate = torch.rand(B * H, S, device=dev, generator=g) + 0.5
    table = torch.randn(H, 2 * S - 1, device=dev, generator=g)
    f = lambda: ops.attn_fwd(qkv, qkv[:, H * 64:], qkv[:, 2 * H * 64:], o, lse, B, H, S, S, gate=gate, table=table)  # noqa
    ms = timeit(f)
    res.append(f"enc fwd {ms*1e3:6.1f} us {4*B*H*S*S*64/ms/1e9:5.0f} TF/s")
    # decoder self (L 256, key mask, dropout 0.1) and cross (L 256 x S 499, dropout)
    B, H, L = 32, 8, 256
    for name, Lk in (("self", L), ("cross", S)):
        q = torch.randn(B * L, H * 64, device=dev, dtype=bf, generator=g)
        kv = torch.randn(B * Lk, 2 * H * 64, device=dev, dtype=bf, generator=g)
        out = torch.empty(B * L, H * 64, device=dev, dtype=bf)
        ls = torch.empty(B * H, L, device=dev)
        kk = (torch.rand(B, Lk, device=dev, generator=g) > 0.2).to(torch.uint8) if name == "self" else None
        bits = ops.drop_bits(B, H, L, Lk, dev)
        f = lambda: ops.attn_fwd(q, kv, kv[:, H * 64:], out, ls, B, H, L, Lk, key_keep=kk, drop_p=0.1, seed=3,  # noqa
                                 rng_stream=1, dbits=bits)
        ms = timeit(f)
        res.append(f"dec {name} fwd {ms*1e3:6.1f} us {4*B*H*L*Lk*64/ms/1e9:5.0f} TF/s")
        do = torch.randn_like(out)
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        fb = lambda: ops.attn_bwd(q, kv, kv[:, H * 64:], out, do, ls, dq, dkv, dkv[:, H * 64:], B, H, L, Lk,  # noqa
                                  key_keep=kk, drop_p=0.1, seed=3, rng_stream=1, dbits=bits)
        ms = timeit(fb)
        res.append(f"dec {name} bwd {ms*1e3:6.1f} us {10*B*H*L*Lk*64/ms/1e9:5.0f} TF/s")
    print(os.path.basename(os.environ.get("FDDM_HIP_LIB", "in-tree")), " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
