"""Micro-benchmark of the fused KL kernels at the C2 shape (B*L = 8192 tokens, V = 8000): HIP-event time per
launch and achieved HBM GB/s (algorithmic bytes: fwd reads the fp32 logits; bwd reads them and writes the bf16
gradient). FDDM_KL_SCALAR=1 selects the scalar-load kernel (read per launch)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402
from oracle import fddm_oracle as O  # noqa: E402


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
    dev = torch.device("cuda:0")
    N, L, V, B = 8192, 256, 8000, 32
    z = 3 * torch.randn(N, V, device=dev)
    xt = torch.randint(1, V, (N,), device=dev)
    x0 = torch.randint(1, V, (N,), device=dev)
    t = torch.randint(1, 201, (B,), device=dev)
    betas = O.sched_tables(200)[0].to(dev)
    w = torch.full((N,), 1.0 / N, device=dev)
    for nt in ("128", "256", "512", "1024"):
        os.environ["FDDM_KLF_NT"] = nt
        tk = timeit(lambda: ops.kl_fused(z, xt, x0, t, betas, None, L, out_dtype=torch.bfloat16))
        print(f"fused fwd+grad NT={nt}: {tk * 1e3:7.1f} us  {(N * V * 6) / tk / 1e6:7.0f} GB/s", flush=True)
    del os.environ["FDDM_KLF_NT"]
    mask = (torch.rand(B, L, device=dev) > 0.2).to(torch.uint8)
    tk = timeit(lambda: ops.kl_fused(z, xt, x0, t, betas, mask, L, out_dtype=torch.bfloat16))
    print(f"fused fwd+grad NT=256 masked: {tk * 1e3:7.1f} us  {(N * V * 6) / tk / 1e6:7.0f} GB/s", flush=True)
    for mode in ("vector", "scalar"):
        if mode == "scalar":
            os.environ["FDDM_KL_SCALAR"] = "1"
        tf = timeit(lambda: ops.kl_fwd(z, xt, x0, t, betas, L))
        tb = timeit(lambda: ops.kl_bwd(z, xt, x0, t, betas, w, None, L, out_dtype=torch.bfloat16))
        print(f"{mode:7s} fwd {tf*1e3:7.1f} us {N*V*4/tf/1e6:7.0f} GB/s | bwd(bf16) {tb*1e3:7.1f} us "
              f"{N*V*6/tb/1e6:7.0f} GB/s", flush=True)
    os.environ.pop("FDDM_KL_SCALAR", None)


if __name__ == "__main__":
    main()
