"""Timing of the 128x128 LDS-DMA GEMM at the decoder's shapes (library chosen by FDDM_HIP_LIB, so two builds can be
compared on one box): dX GEMMs, forward GEMMs forced onto the 128 path, and one decoder block's grouped weight
gradients. HIP-event timing, 20 back-to-back launches after 3 warm-ups."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
GEMM_PATH = "128"   # applied after the import below (ops.gemm_force_path)
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

ops.gemm_force_path(GEMM_PATH)

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
    return s.elapsed_time(e) / iters * 1e3


def main():
    tag = os.path.basename(os.environ.get("FDDM_HIP_LIB", "in-tree"))
    M = 32 * 256
    for (n, k) in [(512, 2048), (2048, 512), (512, 512), (1536, 512)]:
        dy = torch.randn(M, k, device=dev, dtype=bf)
        w = torch.randn(k, n, device=dev, dtype=bf)
        o = torch.empty(M, n, device=dev)
        t = timeit(lambda: ops.linear_dx(dy, w, out=o))
        print(f"[{tag}] dX  {M}x{n}x{k}: {t:7.1f} us {2.0 * M * n * k / t / 1e6:6.0f} TF/s", flush=True)
    for (n, k) in [(1536, 512), (2048, 512), (512, 2048)]:
        x = torch.randn(M, k, device=dev, dtype=bf)
        w = torch.randn(n, k, device=dev, dtype=bf) * 0.02
        t = timeit(lambda: ops.linear(x, w, out_dtype=bf))
        print(f"[{tag}] fwd {M}x{n}x{k}: {t:7.1f} us {2.0 * M * n * k / t / 1e6:6.0f} TF/s", flush=True)
    Me = 32 * 499
    shapes = [(M, 1536, 512), (M, 512, 512), (M, 512, 512), (M, 512, 512), (M, 2048, 512), (M, 512, 2048),
              (Me, 1024, 512)]
    jobs, fl = [], 0.0
    for (m, a, b) in shapes:
        jobs.append((torch.randn(m, a, device=dev, dtype=bf), torch.randn(m, b, device=dev, dtype=bf),
                     torch.zeros(a, b, device=dev), torch.zeros(a, device=dev)))
        fl += 2.0 * m * a * b
    t = timeit(lambda: ops.linear_dw_grouped(jobs))
    print(f"[{tag}] grouped dW of one decoder block ({fl / 1e9:.1f} GFLOP): {t:7.1f} us {fl / t / 1e6:6.0f} TF/s",
          flush=True)


if __name__ == "__main__":
    main()
