"""Fused KL forward + gradient (ops.kl_fused, csrc/kl.hip kl4_fused_kernel) at the C2 train-step shape: B*L = 8192
rows of V = 8000 f32 logits in, bf16 gradient out (393 MB). HIP-event timing of 20 back-to-back launches after 3
warm-ups, against a float4 copy of the same bytes as the achievable-HBM yardstick."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    B, L, V, T = 32, 256, 8000, 200
    N = B * L
    g = torch.Generator(device=dev).manual_seed(0)
    logits = torch.randn(N, V, device=dev, generator=g) * 3
    xt = torch.randint(0, V, (N,), device=dev, generator=g)
    x0 = torch.where(torch.rand(N, device=dev, generator=g) < 0.5, xt, torch.randint(0, V, (N,), device=dev, generator=g))
    t = torch.randint(1, T + 1, (B,), device=dev, generator=g)
    betas = 0.2 * torch.sin(torch.pi * torch.arange(1, T + 1, device=dev) / (2 * T)) ** 2
    mask = (torch.rand(N, device=dev, generator=g) < 0.9).to(torch.uint8)
    us = timeit(lambda: ops.kl_fused(logits, xt, x0, t, betas, mask, L, out_dtype=torch.bfloat16))
    nbytes = N * V * (4 + 2)
    src = torch.empty(nbytes // 2 // 4, device=dev)
    dst = torch.empty_like(src)
    cu = timeit(lambda: dst.copy_(src))
    print(f"kl_fused N={N} V={V}: {us:7.1f} us  {nbytes / us / 1e6:5.2f} TB/s ({nbytes / us / 8e6:.2f} of 8 TB/s) | "
          f"copy of {nbytes / 1e6:.0f} MB: {cu:6.1f} us {nbytes / cu / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
