"""Fixed cost vs K-loop cost of the decoder's d_model-wide GEMMs: ops.linear (ops.gemm_force_path(sys.argv[1]) picks the kernel) at
M = 8192 tokens, N = 512, K = 64 .. 2048, against torch.matmul (hipBLASLt) on the same operands. HIP-event timing,
20 back-to-back launches after 3 warm-ups (tools/g128_bench.py's timer)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

ops.gemm_force_path(sys.argv[1] if len(sys.argv) > 1 else "auto")
from g128_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
M = 8192
for N in (512, 1024, 2048):
    for K in (64, 128, 256, 512, 1024, 2048):
        x = torch.randn(M, K, device=dev, dtype=bf)
        w = torch.randn(N, K, device=dev, dtype=bf) * 0.02
        o = torch.empty(M, N, device=dev, dtype=bf)
        t = timeit(lambda: ops.linear(x, w, out=o))
        tl = timeit(lambda: torch.matmul(x, w.t(), out=o))
        fl = 2.0 * M * N * K
        print(f"[{(sys.argv[1] if len(sys.argv) > 1 else 'auto')}] {M}x{N}x{K}: ours {t:6.1f} us {fl / t / 1e6:5.0f} TF/s | "
              f"hipBLASLt {tl:6.1f} us {fl / tl / 1e6:5.0f} TF/s", flush=True)
