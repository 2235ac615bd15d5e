"""One bf16 GEMM shape of the train step, launched `iters` times through ops.linear (for counter passes).
  python tools/gemm_one.py M N K [iters] [epi]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
epi = int(sys.argv[5]) if len(sys.argv) > 5 else ops.EPI_STORE
dev = torch.device("cuda:0")
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
b = torch.randn(N, device=dev)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3):
    ops.linear(x, w, b, out_dtype=torch.bfloat16, epi=epi)
s.record()
for _ in range(iters):
    ops.linear(x, w, b, out_dtype=torch.bfloat16, epi=epi)
e.record()
torch.cuda.synchronize()
t = s.elapsed_time(e) / iters * 1e3
print(f"M={M} N={N} K={K}: {t:.1f} us, {2.0 * M * N * K / t / 1e6:.0f} TF/s")
