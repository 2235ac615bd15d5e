"""Micro-benchmark of the decoder's small HBM kernels at the C2 shapes (8192 tokens, d 512, V 8000, L 256):
token-embedding forward / backward, RoPE forward / backward. HIP-event timing."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, L, d, V = 32, 256, 512, 8000
    tok = torch.randint(0, V, (B * L,), device=dev)
    dx = torch.randn(B * L, d, device=dev)
    dE = torch.zeros(V, d, device=dev)
    dtb = torch.zeros(B, d, device=dev)
    E = torch.randn(V, d, device=dev)
    tb = torch.randn(B, d, device=dev)
    x = torch.empty(B * L, d, device=dev)
    xt = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
    cos, sin = torch.randn(L, d, device=dev), torch.randn(L, d, device=dev)
    xr = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
    dxr = torch.zeros(B * L, d, device=dev)
    cases = [("embed_bwd", lambda: ops.embed_bwd(tok, dx, dE, dtb, L, 0)),
             ("embed_fwd", lambda: ops.embed_fwd(tok, E, tb, x, xt, L)),
             ("rope_fwd", lambda: ops.rope_fwd(dx, cos, sin, xr, L)),
             ("rope_bwd", lambda: ops.rope_bwd(dx, cos, sin, dxr, L))]
    for name, f in cases:
        for _ in range(5):
            f()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            f()
        e.record()
        torch.cuda.synchronize()
        print(f"{name} {s.elapsed_time(e) / 50 * 1e3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
